"""Where the per-step copies of a model's training step come from: one eager step under
torch.profiler with Python stacks; prints the aten::copy_ / to / contiguous / cat call sites
with their GPU time.   python tools/copy_sites.py [--preset bert_dp8]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="bert_dp8")
    a = ap.parse_args()
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    info = pdist.init_distributed()
    cfg = preset_config(a.preset)
    V = cfg.vocab_hash_size
    tr = Trainer(cfg, build_model(cfg, V), info.device, graph=False)
    data = SyntheticPairs(spec_from_config(cfg, V, num_pages=4096), info.device, seed=1)
    batches = [data.batch(cfg.batch_size) for _ in range(3)]
    for q, d in batches[:2]:
        tr.train_step(q, d)
    torch.cuda.synchronize()
    import traceback

    sites = {}

    def site():
        for fr in reversed(traceback.extract_stack()[:-2]):
            if "dnn_page_vectors_amd" in fr.filename:
                return f"{os.path.relpath(fr.filename, os.path.dirname(os.path.dirname(__file__)))}:{fr.lineno}"
        return "?"

    def wrap(owner, name):
        orig = getattr(owner, name)

        def w(*args, **kw):
            out = orig(*args, **kw)
            t = out if isinstance(out, torch.Tensor) else None
            src = args[0] if args and isinstance(args[0], torch.Tensor) else None
            if t is not None and t.is_cuda and (src is None or t.data_ptr() != src.data_ptr()):
                k = (name, site())
                n, b = sites.get(k, (0, 0))
                sites[k] = (n + 1, b + t.numel() * t.element_size())
            return out
        setattr(owner, name, w)
        return orig

    saved = [(torch.Tensor, n, wrap(torch.Tensor, n)) for n in ("to", "contiguous", "clone", "float", "bfloat16")]
    saved += [(torch, n, wrap(torch, n)) for n in ("cat", "zeros", "zeros_like", "stack")]
    saved += [(torch.Tensor, n, wrap(torch.Tensor, n)) for n in ("zero_", "fill_", "copy_")]
    try:
        tr.train_step(*batches[2])
        torch.cuda.synchronize()
    finally:
        for owner, n, orig in saved:
            setattr(owner, n, orig)
    for (name, where), (n, b) in sorted(sites.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{b / 1e6:9.1f} MB {n:4d}x {name:11s} {where}", flush=True)


if __name__ == "__main__":
    main()
