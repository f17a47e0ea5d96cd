"""Host featurizer throughput (the C++ featurizer gets its own benchmark).

Measures texts/s and output tokens/s of ``data.featurize.Featurizer`` (C++ runtime,
thread pool) for the three feature levels at the reference lengths (config.py:80-91:
char 5000, word 975, ngram 2000 for pages), on synthetic page text, and compares the
pure-Python statement of the rules (``data.text.featurize_py``) on a small sample.

    python tools/featurize_bench.py [--pages 2000] [--threads 0]
"""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dnn_page_vectors_amd.data import text as T  # noqa: E402
from dnn_page_vectors_amd.data.featurize import Featurizer  # noqa: E402
from dnn_page_vectors_amd.data.text import Vocab  # noqa: E402

WORDS = ("statue liberty new york city tour ticket price museum island ferry park hotel "
         "review map history opening hours guide photo family visit harbor bridge").split()


def page(rng: random.Random, n_words: int) -> str:
    return " ".join(rng.choice(WORDS) + (rng.choice(["", "", "!", ",", "'s", " 2019"])) for _ in range(n_words))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pages", type=int, default=2000)
    ap.add_argument("--words", type=int, default=900, help="words per synthetic page (~5.5k chars)")
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args()
    rng = random.Random(0)
    texts = [page(rng, a.words) for _ in range(a.pages)]
    chars = sum(len(t) for t in texts)
    lengths = {"char": 5000, "word": 975, "ngram": 2000}
    for mode, L in lengths.items():
        if mode == "ngram":
            fz = Featurizer(mode, hash_size=30000, nthreads=a.threads)
        else:
            itos = sorted({tok for t in texts[:50] for tok in T.split_features(t, mode)})
            fz = Featurizer(mode, vocab=Vocab(itos), nthreads=a.threads)  # exact-vocab lookup (reference)
        fz(texts[:16], L)  # warm the pool
        t0 = time.perf_counter()
        out = fz(texts, L)
        dt = time.perf_counter() - t0
        ns = min(20, len(texts))
        t1 = time.perf_counter()
        if mode == "ngram":
            T.featurize_py(texts[:ns], mode, L, hash_size=30000)
        else:
            [T.split_features(t, mode) for t in texts[:ns]]
        dpy = (time.perf_counter() - t1) / ns * len(texts)
        print(json.dumps({"mode": mode, "length": L, "pages": len(texts), "threads": fz.nthreads,
                          "pages_per_s": round(len(texts) / dt, 1), "tokens_per_s": round(out.size / dt),
                          "input_MB_per_s": round(chars / dt / 1e6, 1),
                          "python_rules_pages_per_s": round(len(texts) / dpy, 1)}), flush=True)


if __name__ == "__main__":
    main()
