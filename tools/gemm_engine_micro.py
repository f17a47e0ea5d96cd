"""GEMM engine (gemm.hip) vs the library GEMM (torch.mm -> hipBLASLt) at the model shapes,
interleaved in one process on random bf16 operands (cdna_hip_programming.md rule 24/25).

    python tools/gemm_engine_micro.py [--iters 20] [--rounds 3]
Prints one JSON line per shape: median ms and TFLOP/s of both, and the max relative error.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dnn_page_vectors_amd.ops import gemm as gops  # noqa: E402
from dnn_page_vectors_amd.ops._common import lib as _lib  # noqa: E402

L = _lib()

# (name, M, N, K, a_col, b_col): BERT-base at 73728 tokens (B 256 x (32 + 256)), MLP / bag
SHAPES = [
    ("bert_qkv_fwd", 73728, 2304, 768, False, False),
    ("bert_ffn1_fwd", 73728, 3072, 768, False, False),
    ("bert_ffn2_fwd", 73728, 768, 3072, False, False),
    ("bert_ffn2_dgrad", 73728, 3072, 768, False, True),
    ("bert_ffn1_wgrad", 3072, 768, 73728, True, True),
    ("mlp_dense_fwd", 16384, 512, 512, False, False),
    ("square_8192", 8192, 8192, 8192, False, False),
    ("square_4096", 4096, 4096, 4096, False, False),
]


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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = "cuda"
    for name, M, N, K, a_col, b_col in SHAPES:
        if a.only and a.only not in name:
            continue
        A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
        a_ = A.t().contiguous() if a_col else A
        b_ = B.t().contiguous() if b_col else B
        lib_a = a_.t() if a_col else a_          # library: the same storage, as views
        lib_b = b_ if b_col else b_.t()

        def ours():
            return gops.gemm(a_, b_, a_col, b_col)

        def ours_g0():  # the row / column panel tile order (A/B arm)
            L.pv_gemm_set_group(0)
            try:
                return gops.gemm(a_, b_, a_col, b_col)
            finally:
                L.pv_gemm_set_group(4)

        def lib():
            return torch.mm(lib_a, lib_b, out_dtype=torch.float32)

        c1, c2 = ours(), lib()
        err = float((c1 - c2).abs().max() / c2.abs().max())
        err0 = float((ours_g0() - c2).abs().max() / c2.abs().max())
        t1, t2, t3 = [], [], []
        for _ in range(a.rounds):
            t1.append(timeit(ours, a.iters))
            t3.append(timeit(ours_g0, a.iters))
            t2.append(timeit(lib, a.iters))
        m1, m2, m3 = statistics.median(t1), statistics.median(t2), statistics.median(t3)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "a_col": a_col, "b_col": b_col,
                          "ksplit": gops.auto_ksplit(M, N, K), "engine_ms": round(m1, 4),
                          "engine_group0_ms": round(m3, 4), "library_ms": round(m2, 4),
                          "engine_tflops": round(fl / m1 / 1e9, 1), "engine_group0_tflops": round(fl / m3 / 1e9, 1),
                          "library_tflops": round(fl / m2 / 1e9, 1), "max_rel_err": err, "group0_max_rel_err": err0}),
              flush=True)
        del A, B, a_, b_, c1, c2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
