"""Where the per-step copies of a model's training step come from: one eager step under
torch.profiler with Python stacks; prints the aten::copy_ / to / contiguous / cat call sites
with their GPU time.   python tools/copy_sites.py [--preset bert_dp8]"""
import argparse
import os
import sys
from collections import defaultdict

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
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        tr.train_step(*batches[2])
        torch.cuda.synchronize()
    sites = defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::to", "aten::_to_copy", "aten::contiguous", "aten::cat", "aten::clone",
                       "aten::zeros", "aten::fill_", "aten::zero_"):
            stack = [f for f in (ev.stack or []) if "dnn_page_vectors_amd" in f or "bench" in f]
            key = (ev.name, stack[0] if stack else "?")
            sites[key][0] += 1
            sites[key][1] += ev.device_time_total if hasattr(ev, "device_time_total") else ev.cuda_time_total
    rows = sorted(sites.items(), key=lambda kv: -kv[1][1])
    for (name, site), (n, us) in rows[:40]:
        print(f"{us:9.1f} us  {n:4d}x  {name:16s} {site}", flush=True)


if __name__ == "__main__":
    main()
