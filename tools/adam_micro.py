"""Flat-buffer Adam bandwidth: pv_adam (HIP) vs torch.optim.Adam(fused=True) on the same
16 M fp32 parameters (28 bytes moved per parameter).

    python tools/adam_micro.py [--n 16777216] [--lazy-rows 7500000 --lazy-cols 100 --touched 0.01]

--lazy-rows: also time the lazy embedding-row update (pv_adam_seg row_len > 0) on a
(rows, cols) table with a fraction ``--touched`` of rows carrying a gradient, against the
dense update of the same table (a word-level vocabulary of millions of rows).
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


def lazy(a):
    from dnn_page_vectors_amd.ops._common import P, check, lib, stream

    R, C = a.lazy_rows, a.lazy_cols
    n = R * C
    p, m, v = (torch.zeros(n, device="cuda") for _ in range(3))
    g = torch.zeros(R, C, device="cuda")
    rows = torch.randperm(R, device="cuda")[:max(1, int(R * a.touched))]
    g[rows] = torch.randn(rows.numel(), C, device="cuda")
    t = torch.tensor([1.0, 0.0], device="cuda")  # {step, warmup steps}
    L = lib()
    res = {}
    for name, rl in (("dense", 0), ("lazy", C)):
        res[name + "_ms"] = round(ev(lambda: check(L.pv_adam_seg(P(p), P(g), P(m), P(v), n, rl, P(t), 1e-3, 0.9, 0.999,
                                                                  1e-8, 0.0, 0, None, stream()), "seg")), 4)
    print(json.dumps({"rows": R, "cols": C, "touched": a.touched, **res}), flush=True)


def main():
    from dnn_page_vectors_amd.ops._common import P, check, lib, stream

    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16 * 1024 * 1024)
    ap.add_argument("--lazy-rows", type=int, default=0)
    ap.add_argument("--lazy-cols", type=int, default=100)
    ap.add_argument("--touched", type=float, default=0.01)
    a = ap.parse_args()
    if a.lazy_rows:
        lazy(a)
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
