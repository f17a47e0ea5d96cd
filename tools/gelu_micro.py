"""BERT FFN bias + GELU forward / backward kernels (transformer.hip) at T 73728 x 3072:
round-2 vector kernels (pv_gelu_set_v 1) vs the 128-thread unrolled ones (2), CUDA events."""
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
    return round(a.elapsed_time(b) / it * 1000, 1)


def main():
    from dnn_page_vectors_amd.ops._common import P, lib, stream

    dev = torch.device("cuda")
    M, D = 73728, 3072
    x = torch.randn(M, D, device=dev).bfloat16()
    b = torch.randn(D, device=dev)
    y = torch.empty_like(x)
    dy = torch.randn(M, D, device=dev).bfloat16()
    dx = torch.empty_like(x)
    db = torch.empty(D, device=dev)
    ws = torch.empty(lib().pv_bias_gelu_bwd_ws(M, D), device=dev)
    s = stream(dev)
    r = {}
    for rnd in range(2):
        for v in (1, 2, 3):
            lib().pv_gelu_set_v(v)
            r[f"fwd_v{v}_r{rnd}"] = ev(lambda: lib().pv_bias_gelu_fwd(P(x), P(b), P(y), M * D, D, s))
            r[f"bwd_v{v}_r{rnd}"] = ev(lambda: lib().pv_bias_gelu_bwd(P(x), P(b), P(dy), P(dx), P(db), P(ws), M, D, s))
    lib().pv_gelu_set_v(2)
    # add + LayerNorm forward (dropout 0.1, branch bias) at T x 768: rows per wave 1 / 2 / 4
    H = 768
    xa = torch.randn(M, H, device=dev).bfloat16()
    ra = torch.randn(M, H, device=dev).bfloat16()
    g_, b_, xb_ = torch.ones(H, device=dev), torch.zeros(H, device=dev), torch.zeros(H, device=dev)
    ya, ha = torch.empty_like(xa), torch.empty_like(xa)
    mu, rs = torch.empty(M, device=dev), torch.empty(M, device=dev)
    for rnd in range(2):
        for rpw in (1, 2, 4):
            lib().pv_ln_set_rpw(rpw)
            r[f"addln_rpw{rpw}_r{rnd}"] = ev(lambda: lib().pv_add_ln_drop_fwd(
                P(xa), P(xb_), P(ra), P(g_), P(b_), P(ya), P(ha), P(mu), P(rs), M, H, 1e-12, 26, 256.0 / 230, 7, None, s))
    lib().pv_ln_set_rpw(2)
    # LN backward (with the dropout-branch output) with / without the next-row prefetch
    dya = torch.randn(M, H, device=dev).bfloat16()
    dxa, dxm = torch.empty_like(xa), torch.empty_like(xa)
    dgam, dbet, dxb = torch.empty(H, device=dev), torch.empty(H, device=dev), torch.empty(H, device=dev)
    wsl = torch.empty(lib().pv_layernorm_bwd_ws(M, H), device=dev)
    for rnd in range(2):
        for pf in (0, 1):
            lib().pv_ln_bwd_set_pf(pf)
            r[f"lnbwd_pf{pf}_r{rnd}"] = ev(lambda: lib().pv_layernorm_bwd_drop(
                P(dya), P(ha), P(g_), P(mu), P(rs), P(dxa), P(dxm), P(dgam), P(dbet), P(dxb), P(wsl), M, H, 26,
                256.0 / 230, 7, None, s))
    lib().pv_ln_bwd_set_pf(1)
    r["addln_best_TBps"] = round(4 * M * H * 2 / 1e9 / min(v for k, v in r.items() if k.startswith("addln")) * 1e3, 2)
    gb = M * D * 2 / 1e9
    r["fwd_v1_TBps"] = round(2 * gb / min(r["fwd_v1_r0"], r["fwd_v1_r1"]) * 1e6 / 1e3, 2)
    r["bwd_v2_TBps"] = round(3 * gb / min(r["bwd_v2_r0"], r["bwd_v2_r1"]) * 1e6 / 1e3, 2)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
