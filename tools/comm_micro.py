#!/usr/bin/env python3
"""RCCL collective micro-benchmark for the training step's traffic.

Times, at the launch's world size W, the collectives a data-parallel step issues:

* bucketed gradient all-reduce of the CDSSM (13 MB), MLP (126 MB) and BERT-base (440 MB)
  fp32 gradients, cut into buckets of ``--bucket-mb`` (the trainer's ``grad_bucket_mb``),
  all buckets in flight at once as the backward hooks launch them;
* the page-vector all-gather of the cross-GPU loss (B 4096 x 4 pages x 150-d bf16 = 9.8 MB
  per rank at the headline shape) and the query all-gather (2.6 MB);

and prints one JSON line per (collective, size, bucket) with the time, the algorithm
bandwidth (bytes / time) and the ring bus bandwidth (x 2(W-1)/W for all-reduce, x (W-1)/W
for all-gather) — the per-link number to compare with ~153 GB/s per xGMI link.

    python -m dnn_page_vectors_amd.launch --nproc 8 -- tools/comm_micro.py [--bucket-mb 8 32 128]
    tools/comm_micro.py --sweep-channels 4 8 16 32 --nproc 8     (one launch per NCCL_MIN_NCHANNELS)

``--sweep-channels`` starts one launch per value with ``NCCL_MIN_NCHANNELS`` (and
``NCCL_MAX_NCHANNELS``) set, so the first 8-GPU lease yields the tuning table for
``grad_bucket_mb`` and the channel count; bench.py records both in its JSON ``config``.
CPU: ``--device cpu`` runs the same code over gloo (tests / rehearsal).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GRADS_MB = {"cdssm": 12.6, "mlp": 126.0, "bert": 440.0}
GATHER_MB = {"page_vectors": 4096 * 4 * 160 * 2 / 2**20, "queries": 4096 * 160 * 2 / 2**20}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bucket-mb", type=float, nargs="+", default=[8.0, 32.0, 128.0])
    ap.add_argument("--models", nargs="+", default=list(GRADS_MB))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scale", type=float, default=1.0, help="multiply every message size (tests: tiny)")
    ap.add_argument("--device", default=None, help="cuda (RCCL) or cpu (gloo)")
    ap.add_argument("--sweep-channels", type=int, nargs="*", default=None,
                    help="re-launch once per NCCL_MIN_NCHANNELS value (needs --nproc)")
    ap.add_argument("--nproc", type=int, default=0)
    return ap.parse_args()


def sweep(a) -> int:
    from dnn_page_vectors_amd.launch import launch

    rc = 0
    args = [x for x in sys.argv[1:]]
    i = args.index("--sweep-channels")
    j = i + 1
    while j < len(args) and not args[j].startswith("--"):
        j += 1
    rest = args[:i] + args[j:]
    for ch in a.sweep_channels:
        env = dict(os.environ, NCCL_MIN_NCHANNELS=str(ch), NCCL_MAX_NCHANNELS=str(ch))
        rc = rc or launch([sys.executable, os.path.abspath(__file__)] + rest, a.nproc, env=env)
    return rc


def main() -> int:
    a = parse()
    if a.sweep_channels is not None:
        if a.nproc < 1:
            raise SystemExit("--sweep-channels needs --nproc N")
        return sweep(a)
    import torch
    import torch.distributed as dist

    from dnn_page_vectors_amd.parallel import dist as pdist

    info = pdist.init_distributed(device=a.device)
    dev = info.device
    W = info.world_size

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def timed(fn) -> float:
        for _ in range(a.warmup):
            fn()
        sync()
        pdist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        sync()
        dt = torch.tensor([(time.perf_counter() - t0) / a.iters], dtype=torch.float64,
                          device=dev if info.backend == "nccl" else "cpu")
        pdist.all_reduce_max_(dt)
        return float(dt)

    env = {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_")) and "SOCKET" not in k}

    def emit(**kw):
        if info.is_main:
            print(json.dumps(dict(world=W, backend=info.backend, env=env, **kw)), flush=True)

    for m in a.models:
        total = int(GRADS_MB[m] * a.scale * 2**20 / 4)
        g = torch.ones(total, dtype=torch.float32, device=dev)
        for bmb in a.bucket_mb:
            cap = max(1, int(bmb * a.scale * 2**20 / 4))
            views = [g[i:i + cap] for i in range(0, total, cap)]

            def allreduce():
                hs = [dist.all_reduce(v, async_op=True) for v in views]
                for h in hs:
                    h.wait()
            t = timed(allreduce) if W > 1 else 0.0
            nbytes = total * 4
            emit(op="all_reduce", model=m, mbytes=round(nbytes / 2**20, 2), bucket_mb=bmb, buckets=len(views),
                 ms=round(t * 1e3, 4), algbw_gbs=round(nbytes / t / 1e9, 2) if t else None,
                 busbw_gbs=round(nbytes / t / 1e9 * 2 * (W - 1) / W, 2) if t else None)
        del g
    for name, mb in GATHER_MB.items():
        n = max(1, int(mb * a.scale * 2**20 / 2))
        x = torch.ones(n, dtype=torch.bfloat16, device=dev)
        out = torch.empty(W * n, dtype=torch.bfloat16, device=dev)
        t = timed(lambda: dist.all_gather_into_tensor(out, x)) if W > 1 else 0.0
        nbytes = W * n * 2
        emit(op="all_gather", tensor=name, mbytes_per_rank=round(n * 2 / 2**20, 3), ms=round(t * 1e3, 4),
             algbw_gbs=round(nbytes / t / 1e9, 2) if t else None,
             busbw_gbs=round(nbytes / t / 1e9 * (W - 1) / W, 2) if t else None)
    pdist.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
