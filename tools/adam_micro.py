"""Flat-buffer Adam bandwidth: pv_adam (HIP) vs torch.optim.Adam(fused=True) on the same
16 M fp32 parameters (28 bytes moved per parameter).

    python tools/adam_micro.py [--n 16777216]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ev(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    from dnn_page_vectors_amd.ops._common import P, check, lib, stream

    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16 * 1024 * 1024)
    a = ap.parse_args()
    n = a.n
    p, g, m, v = (torch.randn(n, device="cuda") for _ in range(4))
    v.abs_()
    L = lib()
    t_hip = ev(lambda: check(L.pv_adam(P(p), P(g), P(m), P(v), n, 5, 1e-3, 0.9, 0.999, 1e-8, 0.0, 0, None,
                                       stream()), "adam"))
    t_sq = ev(lambda: check(L.pv_sumsq(P(g), n, P(m[:2]), stream()), "sumsq"))
    pt = torch.nn.Parameter(torch.randn(n, device="cuda"))
    pt.grad = torch.randn(n, device="cuda")
    opt = torch.optim.Adam([pt], lr=1e-3, fused=True)
    t_torch = ev(opt.step)
    gb = 28.0 * n / 1e9
    print(json.dumps({"n": n, "pv_adam_ms": round(t_hip, 4), "pv_adam_TBps": round(gb / t_hip, 2),
                      "torch_fused_adam_ms": round(t_torch, 4), "torch_TBps": round(gb / t_torch, 2),
                      "pv_sumsq_ms": round(t_sq, 4), "sumsq_TBps": round(4.0 * n / 1e9 / t_sq, 2)}), flush=True)


if __name__ == "__main__":
    main()
