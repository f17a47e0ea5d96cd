"""Micro-benchmark of the CDSSM conv kernels at the bench shape (one process, CUDA events).

    python tools/conv_micro.py [--N 16384] [--L 2000] [--iters 10]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from dnn_page_vectors_amd.ops import conv_pool as cops


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--L", type=int, default=2000)
    ap.add_argument("--V", type=int, default=30000)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--p", type=float, default=0.25)
    a = ap.parse_args()
    dev = "cuda"
    E, F = 100, 150
    ids = torch.randint(1, a.V, (a.N, a.L), dtype=torch.int32, device=dev)
    table = torch.nn.Parameter(torch.randn(a.V, E, device=dev) * 0.05)
    w3 = torch.nn.Parameter(torch.randn(F, 3, E, device=dev) * 0.05)
    w4 = torch.nn.Parameter(torch.randn(F, 4, E, device=dev) * 0.05)
    b3 = torch.nn.Parameter(torch.zeros(F, device=dev))
    b4 = torch.nn.Parameter(torch.zeros(F, device=dev))
    cache = (cops.table_bf16(table.detach()), cops.pack_weights(w3.detach(), w4.detach()))
    res = {}

    def fwd():
        with torch.no_grad():
            return cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], a.p, 7, True, compute_cache=cache)

    res["fwd_ms"] = timeit(fwd, a.iters)
    flops = 2.0 * a.N * sum((a.L - k + 1) * k * E * F for k in (3, 4))
    res["fwd_tflops_useful"] = flops / (res["fwd_ms"] * 1e-3) / 1e12

    def fwd_bwd():
        pooled, _ = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], a.p, 7, True, compute_cache=cache)
        pooled.backward(torch.ones_like(pooled) * 1e-3)

    res["fwd_bwd_ms"] = timeit(fwd_bwd, a.iters)
    res["bwd_ms"] = res["fwd_bwd_ms"] - res["fwd_ms"]
    res.update(N=a.N, L=a.L, V=a.V)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
