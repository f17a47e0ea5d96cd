"""Retrieval quality after a fixed number of steps (BASELINE.md "Quality"): train a preset on
the synthetic query/page generator and report Recall@1/10/100 on held-out pairs.

    python tools/quality_run.py --preset cdssm_ngram_bf16 --batch 512 --steps 400 --eval-every 100
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dnn_page_vectors_amd.config import preset_config  # noqa: E402
from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config  # noqa: E402
from dnn_page_vectors_amd.eval.retrieval import recall_table  # noqa: E402
from dnn_page_vectors_amd.models import build_model  # noqa: E402
from dnn_page_vectors_amd.parallel import dist as pdist  # noqa: E402
from dnn_page_vectors_amd.train.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="cdssm_ngram_bf16")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--eval-every", type=int, default=100)
    ap.add_argument("--eval-pages", type=int, default=2048)
    ap.add_argument("--lr", type=float, default=0.0)
    ap.add_argument("--loss", default="")
    ap.add_argument("--set", nargs="*", default=[])
    ap.add_argument("--graph", type=int, default=0, help="hipGraph steps")
    ap.add_argument("--graph-fence", type=int, default=0, help="device sync after every replay (Trainer graph_fence)")
    ap.add_argument("--sync-each", action="store_true", help="synchronize + print after every step (debug)")
    ap.add_argument("--no-initial-eval", action="store_true")
    ap.add_argument("--pool", type=int, default=0, help="pre-generate this many batches and cycle them (0 = fresh batch per step)")
    ap.add_argument("--print-each", action="store_true", help="print the step number after each launch (no sync)")
    a = ap.parse_args()
    info = pdist.init_distributed()
    cfg = preset_config(a.preset).replace(batch_size=a.batch)
    if a.lr:
        cfg = cfg.replace(lr=a.lr)
    if a.loss:
        cfg = cfg.replace(loss_mode=a.loss)
    if a.set:
        cfg = cfg.override(a.set)
    V = cfg.vocab_hash_size
    dev = info.device
    data = SyntheticPairs(spec_from_config(cfg, V, num_pages=65536), dev, seed=11)
    model = build_model(cfg, V)
    tr = Trainer(cfg, model, dev, graph=bool(a.graph), graph_fence=bool(a.graph_fence))
    qe, pe = data.eval_set(a.eval_pages)
    rel = torch.arange(a.eval_pages, device=dev)
    t0 = time.time()

    def evaluate(step, loss):
        print(json.dumps({"eval_begin": step}), flush=True)
        r = recall_table(model.encode(qe, "query"), model.encode(pe, "doc"), rel, ks=(1, 10, 100))
        rec = {"preset": a.preset, "step": step, "pairs_seen": step * a.batch, "loss": round(loss, 4),
               **{k: round(v, 4) for k, v in r.items()}, "wall_s": round(time.time() - t0, 1)}
        if os.environ.get("PAGEVEC_DEBUG_KERNELS") == "1":
            from dnn_page_vectors_amd import _native
            rec["debug"] = _native.debug_status()
        print(json.dumps(rec), flush=True)

    if not a.no_initial_eval:
        evaluate(0, float("nan"))
    pool = [data.batch(a.batch) for _ in range(a.pool)]
    for s in range(1, a.steps + 1):
        q, d = pool[s % a.pool] if pool else data.batch(a.batch)
        m = tr.train_step(q, d)
        if a.sync_each:
            torch.cuda.synchronize()
            rec = {"step": s, "ok": True, "graph": tr._graph is not None}
            if os.environ.get("PAGEVEC_DEBUG_KERNELS") == "1":
                from dnn_page_vectors_amd import _native
                rec["debug"] = _native.debug_status()
            print(json.dumps(rec), flush=True)
        elif a.print_each:
            print(json.dumps({"launched": s}), flush=True)
        if s % a.eval_every == 0 or s == a.steps:
            evaluate(s, float(m["loss"]))


if __name__ == "__main__":
    main()
