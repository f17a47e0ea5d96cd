"""Long-bag products of the MLP / chunked towers: in-tree bag_gemm.hip (segment lists +
on-the-fly-count MFMA products) against the library plan (dense bf16 count matrix + hipBLASLt),
on synthetic Zipf pages of the bench distribution.  CUDA-event timed, same process.

    python tools/bag_gemm_micro.py [--N 4096] [--L 2000] [--V 30000] [--E 512]

Reported per call (ms): rle (segment lists), hip_fwd (partials), hip_wgrad, lib_counts (dense
count matrix), lib_fwd (split-K bmm), lib_wgrad (C^T G), dense_fwd / dense_wgrad (the same count
matrix on bagd_mm_kernel, PAGEVEC_BAG_GEMM=dense); plus max relative differences.
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
    rle = eops._Rle(ids, a.V, 0)
    r["rle"] = ev(lambda: eops._Rle(ids, a.V, 0))
    part = rle.forward_partials(W16)
    r["hip_fwd"] = ev(lambda: rle.forward_partials(W16))
    dW = torch.empty(a.V, a.E, device=dev)
    r["hip_wgrad"] = ev(lambda: rle.weight_grad(G16, dW, False))
    C, lens = eops._counts(ids, a.V, 0)
    r["lib_counts"] = ev(lambda: eops._counts(ids, a.V, 0))
    ref = eops._counts_gemm(C[:, :a.V], W16)
    r["lib_fwd"] = ev(lambda: eops._counts_gemm(C[:, :a.V], W16))
    Ct = C[:, :a.V].t()
    out = torch.empty(a.V, a.E, device=dev)
    r["lib_wgrad"] = ev(lambda: torch.mm(Ct, G16, out_dtype=torch.float32, out=out))
    r["fwd_rel_diff"] = float((part.sum(0) - ref).abs().max() / ref.abs().max())
    # the dense-count in-tree arm (PAGEVEC_BAG_GEMM=dense): same count matrix, bagd_mm_kernel
    from dnn_page_vectors_amd.ops import dense as dops
    dref = dops.colsum(eops._dense_forward_partials(C, W16, a.V))
    r["dense_fwd"] = ev(lambda: dops.colsum(eops._dense_forward_partials(C, W16, a.V)))
    out2 = torch.empty(a.V, a.E, device=dev)
    r["dense_wgrad"] = ev(lambda: eops._dense_weight_grad(C, G16, a.V, out2))
    r["dense_fwd_rel_diff"] = float((dref - ref).abs().max() / ref.abs().max())
    from dnn_page_vectors_amd.ops._common import lib
    if os.environ.get("BAG_MICRO_DBG") == "1":  # round-5 timing ablations (bag_gemm.hip DBG bits;
        # wrong results by design — a round-6 run of them faulted, so they are opt-in)
        for d in (1, 2, 3, 4, 8, 12, 15):
            lib().pv_bag_set_dbg(d)
            r[f"fwd_dbg{d}"] = ev(lambda: rle.forward_partials(W16))
        lib().pv_bag_set_dbg(0)
    r["wgrad_rel_diff"] = float((dW - out).abs().max() / out.abs().max())
    r["dense_wgrad_rel_diff"] = float((out2 - out).abs().max() / out.abs().max())
    flops = 2.0 * a.N * a.V * a.E
    r["hip_fwd_tflops"] = round(flops / r["hip_fwd"] / 1e9, 1)
    r["hip_wgrad_tflops"] = round(flops / r["hip_wgrad"] / 1e9, 1)
    r["nnz_per_page"] = float(rle.ao[-1]) / a.N
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
