"""Long-bag products of the MLP / chunked towers on the dense bf16 count matrix: in-tree
bag_gemm.hip (bagd_mm_kernel) against hipBLASLt, on synthetic Zipf pages of the bench
distribution.  CUDA-event timed, same process.

    python tools/bag_gemm_micro.py [--N 4096] [--L 2000] [--V 30000] [--E 512]

Reported per call (ms): lib_counts (dense count matrix), lib_fwd (split-K bmm), lib_wgrad
(C^T G), dense_fwd / dense_wgrad (the same count matrix on bagd_mm_kernel,
PAGEVEC_BAG_GEMM=dense); plus max relative differences.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def ev(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / it, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--L", type=int, default=2000)
    ap.add_argument("--V", type=int, default=30000)
    ap.add_argument("--E", type=int, default=512)
    a = ap.parse_args()
    from dnn_page_vectors_amd.config import Configuration
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.ops import embedding as eops

    dev = torch.device("cuda")
    cfg = Configuration(feature_level="ngram", vocab_hash_size=a.V, query_length=45, document_length=a.L, J=0)
    data = SyntheticPairs(spec_from_config(cfg, a.V, num_pages=a.N), dev, seed=5)
    ids = data.pages[:a.N].contiguous()
    W16 = torch.randn(a.V, a.E, device=dev).bfloat16()
    G16 = torch.randn(a.N, a.E, device=dev).bfloat16()
    r = {"shape": [a.N, a.L, a.V, a.E]}
    C, lens = eops._counts(ids, a.V, 0)
    r["lib_counts"] = ev(lambda: eops._counts(ids, a.V, 0))
    ref = eops._counts_gemm(C[:, :a.V], W16)
    r["lib_fwd"] = ev(lambda: eops._counts_gemm(C[:, :a.V], W16))
    Ct = C[:, :a.V].t()
    out = torch.empty(a.V, a.E, device=dev)
    r["lib_wgrad"] = ev(lambda: torch.mm(Ct, G16, out_dtype=torch.float32, out=out))
    # the dense-count in-tree arm (PAGEVEC_BAG_GEMM=dense): same count matrix, bagd_mm_kernel
    from dnn_page_vectors_amd.ops import dense as dops
    dref = dops.colsum(eops._dense_forward_partials(C, W16, a.V))
    r["dense_fwd"] = ev(lambda: dops.colsum(eops._dense_forward_partials(C, W16, a.V)))
    out2 = torch.empty(a.V, a.E, device=dev)
    r["dense_wgrad"] = ev(lambda: eops._dense_weight_grad(C, G16, a.V, out2))
    r["dense_fwd_rel_diff"] = float((dref - ref).abs().max() / ref.abs().max())
    r["dense_wgrad_rel_diff"] = float((out2 - out).abs().max() / out.abs().max())
    flops = 2.0 * a.N * a.V * a.E
    r["dense_fwd_tflops"] = round(flops / r["dense_fwd"] / 1e9, 1)
    r["dense_wgrad_tflops"] = round(flops / r["dense_wgrad"] / 1e9, 1)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
