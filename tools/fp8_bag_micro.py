"""Config-5 page bag (fp8 forward) forward + backward: weight gradient on the MX fp8 MFMA
(PAGEVEC_FP8_BWD=1: e4m3 counts^T x e4m3 dz/len) vs the exact bf16 counts + hipBLASLt C^T G,
CUDA-event timed in one process, plus the pieces of the fp8 weight gradient.

    python tools/fp8_bag_micro.py [--N 4096] [--L 512] [--V 30000] [--E 512]
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
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--V", type=int, default=30000)
    ap.add_argument("--E", type=int, default=512)
    a = ap.parse_args()
    from dnn_page_vectors_amd.config import Configuration
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.ops import embedding as eops
    from dnn_page_vectors_amd.ops import fp8 as fops
    from dnn_page_vectors_amd.ops._common import P, lib, stream

    dev = torch.device("cuda")
    cfg = Configuration(feature_level="ngram", vocab_hash_size=a.V, query_length=45, document_length=a.L, J=0)
    data = SyntheticPairs(spec_from_config(cfg, a.V, num_pages=a.N), dev, seed=5)
    ids = data.pages[:a.N].contiguous()
    W = (torch.randn(a.V, a.E, device=dev) * 0.05).requires_grad_(True)
    b = torch.zeros(a.E, device=dev, requires_grad=True)
    gy = torch.randn(a.N, a.E, device=dev)
    r = {"shape": [a.N, a.L, a.V, a.E]}

    def step():
        W.grad = None
        b.grad = None
        y = eops.embedding_bag(ids, W, pad=0, mean=True, plan="counts", act="tanh", fp8=True, bias=b)
        y.backward(gy)
    for rnd in range(2):
        for arm in (False, True):
            eops.FP8_BWD = arm
            r[f"fwd_bwd_fp8bwd{int(arm)}_r{rnd}"] = ev(step)
    # pieces of the fp8 weight gradient
    Np = -(-a.N // fops.MX_BK) * fops.MX_BK
    C8, _, lens = eops._counts8(ids, a.V, 0, False)
    dz = torch.randn(a.N, a.E, device=dev)
    r["quantize_t"] = ev(lambda: fops.quantize_t(dz, Np))
    ct = torch.empty(a.V, Np, dtype=torch.uint8, device=dev)
    r["transpose_u8"] = ev(lambda: lib().pv_transpose_u8(P(C8), C8.stride(0), a.N, a.V, P(ct), Np, stream(dev)))
    g8t, amax = fops.quantize_t(dz, Np)
    out = torch.empty(a.V, a.E, device=dev)
    r["gemm_mx8_wgrad"] = ev(lambda: lib().pv_gemm_mx8(P(ct), Np, P(g8t), Np, P(out), a.E, a.V, a.E, Np, 1, 0, None,
                                                       1.0 / fops.FP8_MAX, P(amax), 0, 0, stream(dev)))
    C8b, C16, _ = eops._counts8(ids, a.V, 0, True)
    r["counts8_with_bf16"] = ev(lambda: eops._counts8(ids, a.V, 0, True))
    r["counts8_only"] = ev(lambda: eops._counts8(ids, a.V, 0, False))
    gs = dz.bfloat16()
    o2 = torch.empty(a.V, a.E, device=dev)
    r["bf16_wgrad_mm"] = ev(lambda: torch.mm(C16[:, :a.V].t(), gs, out_dtype=torch.float32, out=o2))
    r["wgrad_tflops_fp8"] = round(2.0 * a.N * a.V * a.E / r["gemm_mx8_wgrad"] / 1e9, 1)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
