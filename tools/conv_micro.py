"""Micro-benchmark of the CDSSM conv kernels at the bench shape (one process, CUDA events).

Variants (pv_conv_set_dbg) are timed interleaved in ONE process (cross-process and
cross-device variance would otherwise swamp the deltas — cdna_hip_programming.md §5.4
rule 24).  Bits: 1 no gather, 2 max-only epilogue, 4 no dropout hash, 8 no A-fragment
LDS reads, 16 A prefetch depth 2.

    python tools/conv_micro.py [--N 16384] [--L 2000] [--variants 0,16,7] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from dnn_page_vectors_amd.ops import conv_pool as cops
from dnn_page_vectors_amd.ops._common import lib


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
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--p", type=float, default=0.25)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--bwd", action="store_true")
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
    flops = 2.0 * a.N * sum((a.L - k + 1) * k * E * F for k in (3, 4))

    def fwd():
        with torch.no_grad():
            return cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], a.p, 7, True, compute_cache=cache)

    def fwd_bwd():
        pooled, _ = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], a.p, 7, True, compute_cache=cache)
        pooled.backward(torch.ones_like(pooled) * 1e-3)

    variants = [int(v) for v in a.variants.split(",")]
    # schedule variants (>= 256) must reproduce the production kernel bit for bit
    lib().pv_conv_set_dbg(0)
    ref_p, ref_a = fwd()
    for v in variants:
        if v >= 256:
            lib().pv_conv_set_dbg(v)
            pv_, av_ = fwd()
            print(json.dumps({"variant": v, "pooled_maxdiff": float((pv_ - ref_p).abs().max()),
                              "argmax_mismatch": int((av_ != ref_a).sum())}))
    lib().pv_conv_set_dbg(0)
    res = {v: [] for v in variants}
    resb = []
    for r in range(a.rounds):
        for v in variants:
            lib().pv_conv_set_dbg(v)
            res[v].append(timeit(fwd, a.iters))
        lib().pv_conv_set_dbg(0)
        if a.bwd:
            resb.append(timeit(fwd_bwd, a.iters) - timeit(fwd, a.iters))
    lib().pv_conv_set_dbg(0)
    for v in variants:
        ms = statistics.median(res[v])
        print(json.dumps({"variant": v, "fwd_ms_median": round(ms, 3), "fwd_ms_min": round(min(res[v]), 3),
                          "useful_tflops": round(flops / (ms * 1e-3) / 1e12, 1)}))
    if resb:
        print(json.dumps({"bwd_ms_median": round(statistics.median(resb), 3)}))


if __name__ == "__main__":
    main()
