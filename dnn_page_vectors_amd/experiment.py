"""Experiment workspace setup (reference dssm_cnn_v2/setup_experiment.py).

* ``create_workspace``   — data/model/pickled_files/vectors directories (:42-48);
* ``import_dataset``     — copy (or link) a local dataset file into ``input_dataset``; the
  reference downloads from S3 with the aws CLI (:51-59) — there is no network on the
  MI355X box, so the source is a local path;
* ``split_dataset_file`` — 80/20 random split seeded with 1337 (:17-40).  The reference
  samples indices from ``range(0, num_lines + 1)`` (one past the end); here
  ``range(num_lines)``, so exactly ``int(n * (1 - split)) + 1`` rows go to training;
* ``build_vocabulary``   — exact vocabulary over train+val files, saved as JSON.
"""
from __future__ import annotations

import logging
import os
import random
import shutil
from typing import Optional, Tuple

from .config import Configuration
from .utils.fs import count_lines, create_dir

log = logging.getLogger(__name__)


class SetupExperiment:
    def __init__(self, cfg: Optional[Configuration] = None, seed: int = 1337):
        self.conf = cfg or Configuration()
        self.rng = random.Random(seed)

    def create_workspace(self) -> None:
        for d in (self.conf.data_path, self.conf.data_dir, self.conf.trained_model_dir, self.conf.pickle_files_dir,
                  self.conf.vectors_directory):
            create_dir(d)

    def import_dataset(self, source: str, link: bool = False) -> str:
        create_dir(self.conf.data_dir)
        dst = self.conf.input_dataset
        if os.path.abspath(source) != os.path.abspath(dst):
            if link:
                if os.path.lexists(dst):
                    os.remove(dst)
                os.symlink(os.path.abspath(source), dst)
            else:
                shutil.copyfile(source, dst)
        return dst

    def split_dataset_file(self, input_dataset_file: Optional[str] = None) -> Tuple[int, int]:
        src = input_dataset_file or self.conf.input_dataset
        tr, va = self.conf.model_training_data, self.conf.model_validation_data
        if os.path.exists(tr) or os.path.exists(va):
            log.info("input data already split into training and validation sets")
            return count_lines(tr), count_lines(va)
        n = count_lines(src)
        n_train = min(n, int(n * (1 - self.conf.train_validation_split)) + 1)
        train_idx = set(self.rng.sample(range(n), n_train))
        nt = nv = 0
        with open(src, "r", encoding="utf-8") as f, open(tr, "w", encoding="utf-8") as ft, \
                open(va, "w", encoding="utf-8") as fv:
            for i, line in enumerate(f):
                if i in train_idx:
                    ft.write(line.strip() + "\n")
                    nt += 1
                else:
                    fv.write(line.strip() + "\n")
                    nv += 1
        return nt, nv

    def build_vocabulary(self):
        from .data.featurize import generate_vocabulary
        from .io.vocab import save_vocab

        v = generate_vocabulary(self.conf.input_file_list, self.conf.feature_level, self.conf.num_negative_examples,
                                html=self.conf.html_normalize)
        save_vocab(v, self.conf)
        return v
