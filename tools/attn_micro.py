"""BERT attention (attention.hip) forward + backward at the config-4 shapes (pages N 256 x L 256,
queries N 256 x L 32, H 12, d 64) per 16-row-group setting (pv_attn_set_qg), CUDA-event timed.
    python tools/attn_micro.py"""
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
    return round(a.elapsed_time(b) / it * 1000, 1)  # us


def main():
    from dnn_page_vectors_amd.ops._common import P, lib, stream

    dev = torch.device("cuda")
    H = 12
    res = {}
    for N, L in ((256, 256), (256, 32)):
        qkv = (torch.randn(N, L, 3 * H * 64, device=dev) * 0.5).bfloat16()
        mask = torch.ones(N, L, dtype=torch.int32, device=dev)
        mask[:, L - L // 8:] = 0
        out = torch.empty(N, L, H * 64, dtype=torch.bfloat16, device=dev)
        lse = torch.empty(N, H, L, device=dev)
        dout = torch.randn_like(out)
        D = torch.empty(N, H, L, device=dev)
        dqkv = torch.empty_like(qkv)
        s = stream(dev)
        fwd = lambda: lib().pv_attn_fwd(P(qkv), P(mask), P(out), P(lse), N, L, H, 0.125, s)  # noqa: E731
        bwd = lambda: lib().pv_attn_bwd(P(qkv), P(mask), P(out), P(dout), P(lse), P(D), P(dqkv), N, L, H,  # noqa
                                        0.125, s)
        for qg in (1, 2, 4):
            for rnd in range(2):
                lib().pv_attn_set_qg(qg, qg, qg)
                res[f"L{L}_qg{qg}_fwd_r{rnd}"] = ev(fwd)
                res[f"L{L}_qg{qg}_bwd_r{rnd}"] = ev(bwd)
        for qg in (1, 2):
            for rnd in range(2):
                lib().pv_attn_set_qg(qg, qg, qg)
                lib().pv_attn_set_fwd_dma(1)
                res[f"L{L}_qg{qg}_fwd_dma_r{rnd}"] = ev(fwd)
            lib().pv_attn_set_fwd_dma(0)
        for qf, qq, qk in ((1, 1, 2), (1, 2, 1), (2, 1, 1), (4, 1, 1), (1, 4, 1), (1, 1, 4)):
            lib().pv_attn_set_qg(qf, qq, qk)
            res[f"L{L}_bwd_dq{qq}_dkdv{qk}"] = ev(bwd)
        lib().pv_attn_set_qg(0, 0, 0)
        flops = 4.0 * N * H * L * L * 64
        best = min(v for k, v in res.items() if k.startswith(f"L{L}_") and "_fwd_" in k)
        res[f"L{L}_best_fwd_tflops"] = round(flops / best / 1e6, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
