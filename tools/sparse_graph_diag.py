"""Which run diverges in the world-1 RCCL graph test's row-sparse CDSSM arm: eager twice, graph
twice, per-step max |grad difference| against the first eager run (and the first diverging
step).  Run as its own process (it builds a world-1 nccl group):

    PAGEVEC_FORCE_DIST=1 python tools/sparse_graph_diag.py [--steps 22] [--qstream 1]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
os.environ.setdefault("PAGEVEC_FORCE_DIST", "1")
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=22)
    ap.add_argument("--runs", default="e,e,g,g")
    ap.add_argument("--burn", type=int, default=0, help="throwaway eager trainers run first (first-run effects)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="configuration overrides (bisecting the row-sparse / lazy-Adam / query-stream arms)")
    a = ap.parse_args()
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    info = pdist.init_distributed()
    dev = info.device
    cfg = preset_config("cdssm_ngram_bf16").replace(batch_size=64, document_length=256, grad_bucket_mb=1.0,
                                                    sparse_embedding_grad=True, lazy_embedding_adam=True)
    if a.set:
        cfg = cfg.override(a.set)
    print("config:", {k: getattr(cfg, k) for k in ("sparse_embedding_grad", "lazy_embedding_adam", "query_stream")},
          "force_dist:", os.environ.get("PAGEVEC_FORCE_DIST"), flush=True)
    data = SyntheticPairs(spec_from_config(cfg, cfg.vocab_hash_size, num_pages=1024), dev, seed=3)
    batches = [data.batch(cfg.batch_size) for _ in range(a.steps)]
    for _ in range(a.burn):
        torch.manual_seed(1234)
        tb = Trainer(cfg, build_model(cfg, cfg.vocab_hash_size), dev, graph=False)
        for q, d in batches:
            tb.train_step(q, d)
        torch.cuda.synchronize()
        del tb
    ref = None
    for i, kind in enumerate(a.runs.split(",")):
        torch.manual_seed(1234)
        tr = Trainer(cfg, build_model(cfg, cfg.vocab_hash_size), dev, graph=(kind == "g"))
        grads, losses = [], []
        for q, d in batches:
            m = tr.train_step(q, d)
            losses.append(float(m["loss"]))
            grads.append(tr.flat.grad.detach().clone())
        torch.cuda.synchronize()
        if ref is None:
            ref = (grads, losses)
            print(f"run {i} ({kind}): reference", flush=True)
            continue
        diffs = [float((g - r).abs().max() / r.abs().max().clamp(min=1e-30)) for g, r in zip(grads, ref[0])]
        first = next((k for k, x in enumerate(diffs) if x > 1e-3), None)
        # where in the flat gradient the first diverging step differs
        where = ""
        if first is not None:
            dlt = (grads[first] - ref[0][first]).abs()
            idx = int(dlt.argmax())
            names = [(n, o, k) for n, (o, k, _) in tr.flat.offsets.items() if o <= idx < o + k]
            where = f" at flat[{idx}] in {names[0][0] if names else '?'}"
        print(f"run {i} ({kind}): max grad_rel {max(diffs):.3g}, first step > 1e-3: {first}{where}, "
              f"loss_rel {max(abs(x - y) / max(1.0, abs(y)) for x, y in zip(losses, ref[1])):.3g}", flush=True)
    pdist.destroy()


if __name__ == "__main__":
    main()
