"""MX fp8 GEMM engine (csrc/kernels/gemm_mx8.hip) vs hipBLASLt, and the chunk bag forward
(counts + GEMM + mean / bias / tanh epilogue) in bf16 vs fp8.

    python tools/mx8_micro.py [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dnn_page_vectors_amd.ops import embedding as eops  # noqa: E402
from dnn_page_vectors_amd.ops import fp8 as fops  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters):
        st.record()
        fn()
        en.record()
        torch.cuda.synchronize()
        ts.append(st.elapsed_time(en))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for M, N, K in [(4096, 512, 30080), (4096, 4096, 4096), (8192, 8192, 8192), (16384, 512, 30080)]:
        A = torch.randn(M, K, device=dev, generator=g)
        B = torch.randn(N, K, device=dev, generator=g)
        a8 = fops.emulate_e4m3(A).to(torch.float8_e4m3fn).view(torch.uint8)
        b8 = fops.emulate_e4m3(B).to(torch.float8_e4m3fn).view(torch.uint8)
        A16, B16 = A.bfloat16(), B.bfloat16()
        del A, B
        fl = 2.0 * M * N * K
        rec = {"M": M, "N": N, "K": K}
        for ks in sorted({fops.mx8_ksplit(M, N, K), 1}):
            t = timeit(lambda: fops.gemm_mx8(a8, b8, ksplit=ks), a.iters)
            rec[f"mx8_ks{ks}_ms"] = round(t, 4)
            rec[f"mx8_ks{ks}_pflops"] = round(fl / t / 1e12, 3)
        t = timeit(lambda: torch.mm(A16, B16.t()), a.iters)
        rec["hipblaslt_bf16_ms"] = round(t, 4)
        rec["hipblaslt_bf16_pflops"] = round(fl / t / 1e12, 3)
        try:
            af, bf = a8.view(torch.float8_e4m3fn), b8.view(torch.float8_e4m3fn)
            one = torch.ones((), device=dev)
            t = timeit(lambda: torch._scaled_mm(af, bf.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16),
                       a.iters)
            rec["scaled_mm_fp8_ms"] = round(t, 4)
            rec["scaled_mm_fp8_pflops"] = round(fl / t / 1e12, 3)
        except Exception as e:  # noqa: BLE001
            rec["scaled_mm_fp8"] = f"unavailable: {type(e).__name__}"
        print(json.dumps(rec), flush=True)
        del a8, b8, A16, B16
        torch.cuda.empty_cache()
    # the chunk bag forward of config 5 (4096 chunks x 512 ids, V 30000, E 512)
    V, E, N, L = 30000, 512, 4096, 512
    ranks = torch.arange(1, V, dtype=torch.float64, device=dev)
    p = (1.0 / ranks) / (1.0 / ranks).sum()
    ids = (torch.multinomial(p, N * L, replacement=True, generator=g) + 1).view(N, L).to(torch.int32)
    W = torch.randn(V, E, device=dev, generator=g) * 0.05
    b = torch.zeros(E, device=dev)
    W16 = W.bfloat16()
    w8 = fops.quantize_t(W, -(-V // fops.MX_BK) * fops.MX_BK)
    t16 = timeit(lambda: eops.embedding_bag(ids, W, W16, 0, True, "counts", b, "tanh"), a.iters)
    t8 = timeit(lambda: eops.embedding_bag(ids, W, W16, 0, True, "counts", b, "tanh", fp8=True, w8=w8), a.iters)
    tq = timeit(lambda: fops.quantize_t(W, -(-V // fops.MX_BK) * fops.MX_BK), a.iters)
    print(json.dumps({"bag_fwd_bf16_ms": round(t16, 4), "bag_fwd_fp8_ms": round(t8, 4),
                      "quantize_t_ms_per_step": round(tq, 4)}), flush=True)


if __name__ == "__main__":
    main()
