"""Filesystem helpers.

Equivalents of the parts of ``utils/gen_utils.py`` the training path uses:
``create_dir`` (gen_utils.py:53-56), ``get_current_date_time`` (:135-142),
``group_list_concurrency`` (:120-132) and ``split_combined_file`` (:164-195).
"""
from __future__ import annotations

import math
import os
from datetime import datetime
from typing import List, Sequence, TypeVar

T = TypeVar("T")


def create_dir(dir_name: str) -> None:
    """Create ``dir_name`` recursively if it does not exist."""
    os.makedirs(dir_name, exist_ok=True)


def get_current_date_time() -> str:
    """Timestamp string ``%Y-%m-%dT%H-%M-%S`` (gen_utils.py:135-142)."""
    return datetime.today().strftime("%Y-%m-%dT%H-%M-%S")


def group_list_concurrency(items: Sequence[T], n: int) -> List[Sequence[T]]:
    """Split ``items`` into consecutive chunks of ``n`` (last may be shorter)."""
    return [items[i * n:(i + 1) * n] for i in range(int(math.ceil(len(items) / float(n))))]


def split_combined_file(combined_file: str, num_splits: int, tpl: str) -> List[str]:
    """Split a text file into ``num_splits`` roughly equal line ranges ``tpl.format(i)``."""
    with open(combined_file, "rb") as f:
        num_lines = sum(1 for _ in f)
    per = num_lines // num_splits + 1
    out: List[str] = []
    with open(combined_file, "rb") as f:
        fw = None
        for i, line in enumerate(f):
            if i % per == 0:
                if fw:
                    fw.close()
                out.append(tpl.format(len(out)))
                fw = open(out[-1], "wb")
            fw.write(line)
        if fw:
            fw.close()
    return out


def count_lines(path: str) -> int:
    with open(path, "rb") as f:
        return sum(1 for _ in f)
