"""Offline ETL: gold-pair collectors and the page-text join (reference data_collection/*).

The reference scripts run at module level against files (and a private page index,
``cache.db.sm.SM``, that is not in the repo).  These are the same transformations as
pure functions over records, so they are testable and composable:

* ``collect_assessment``  — UCrawl assessment JSON (collect_training_data_assessment.py:47-92):
  Vital/Useful/Relevant/Slightly relevant -> positive; Off-topic/Not found -> negative;
  Foreign language skipped; negatives topped up to 3 with random other URLs.  The
  reference builds 3 rows but, through an indentation slip, emits only the last one
  (:82-89); here all rows are emitted.
* ``collect_type1``       — cliqz type-1 rows {q, doc_corr{url: text}, doc_incorr{url: text}}
  (collect_training_data_type1.py:20-53); also yields text training rows directly.
* ``collect_type3``       — Google type-3 TSV ``query \\t url url ...``: each positive gives 3
  rows with 3 random negatives (collect_training_data_type3.py:41-76).
* ``page_text`` / ``join_pages`` — the join the reference leaves out of the repo (SURVEY
  E5): URL rows + page records ``{url_words, title, desc, top_n_q}``
  (page_info_collector.py:127-143) -> ``{'q', 'doc_corr', 'doc_incorr'}`` training lines.
"""
from __future__ import annotations

import json
import random
from typing import Dict, Iterable, Iterator, List, Optional, Sequence

ASSESSMENTS = ['Vital', 'Useful', 'Relevant', 'Slightly relevant', 'Off-topic / Useless', 'Foreign language',
               'Not found']


def _top_up(negs: List[str], exclude: set, pool: Sequence[str], rng: random.Random, k: int = 3,
            tries: int = 8) -> List[str]:
    out = list(negs)
    for u in rng.sample(list(pool), min(tries, len(pool))):
        if len(out) >= k:
            break
        if u not in exclude and u not in out:
            out.append(u)
    return out


def collect_assessment(records: Iterable[dict], rng: Optional[random.Random] = None, num_neg: int = 3
                       ) -> Iterator[dict]:
    rng = rng or random.Random(1337)
    records = list(records)
    pool = sorted({it["url"] for r in records for it in r["results"]})
    for r in records:
        ranked = sorted(((it["url"], ASSESSMENTS.index(it["assessment"])) for it in r["results"]),
                        key=lambda x: x[1])
        corr = [u for u, a in ranked if a < 4]
        incorr = [u for u, a in ranked if a > 3 and a != 5]
        for u in corr:
            reps = 1 if len(incorr) == num_neg else 3
            for _ in range(reps):
                yield {"q": r["query"], "corr_url": u,
                       "incorr_url": _top_up(incorr[:num_neg], set(corr) | set(incorr), pool, rng, num_neg)}


def collect_type1(records: Iterable[dict], as_text: bool = False) -> Iterator[dict]:
    for r in records:
        corr = next(iter(r["doc_corr"].items()), ("", ""))
        if as_text:
            yield {"q": r["q"], "doc_corr": corr[1], "doc_incorr": list(r["doc_incorr"].values())}
        else:
            yield {"q": r["q"], "corr_url": corr[0], "incorr_url": list(r["doc_incorr"].keys())}


def collect_type3(lines: Iterable[str], rng: Optional[random.Random] = None, num_neg: int = 3,
                  reps: int = 3) -> Iterator[dict]:
    rng = rng or random.Random(1337)
    rows = []
    for line in lines:
        parts = line.rstrip("\n").split("\t")
        if len(parts) == 2:
            rows.append((parts[0], parts[1].split(" ")))
    pool = sorted({u for _, us in rows for u in us})
    for q, corr in rows:
        for u in corr:
            for _ in range(reps):
                yield {"q": q, "corr_url": u, "incorr_url": _top_up([], set(corr), pool, rng, num_neg, tries=10)}


def page_text(info: dict, use_queries: bool = False) -> str:
    """Document text of a page record: title + description + URL words (+ top queries)."""
    parts = [info.get("title", ""), info.get("desc", ""), info.get("url_words", "")]
    if use_queries:
        parts += list(info.get("top_n_q", []))
    return " ".join(p for p in parts if p)


def read_page_info_tsv(lines: Iterable[str]) -> Dict[str, dict]:
    """``json(url) \\t json(record)`` lines (page_info_collector.py:143) -> {url: record}."""
    out = {}
    for line in lines:
        if "\t" not in line:
            continue
        u, rec = line.rstrip("\n").split("\t", 1)
        out[json.loads(u)] = json.loads(rec)
    return out


def join_pages(url_rows: Iterable[dict], pages: Dict[str, dict], num_neg: int = 3,
               use_queries: bool = False) -> Iterator[dict]:
    """{q, corr_url, incorr_url} + page records -> {q, doc_corr, doc_incorr} (pages must exist)."""
    for r in url_rows:
        if r["corr_url"] not in pages:
            continue
        negs = [pages[u] for u in r["incorr_url"] if u in pages]
        if len(negs) != num_neg:
            continue
        yield {"q": r["q"], "doc_corr": page_text(pages[r["corr_url"]], use_queries),
               "doc_incorr": [page_text(n, use_queries) for n in negs]}


def write_jsonl(rows: Iterable[dict], path: str) -> int:
    n = 0
    with open(path, "w", encoding="utf-8") as f:
        for r in rows:
            f.write(json.dumps(r, ensure_ascii=False) + "\n")
            n += 1
    return n
