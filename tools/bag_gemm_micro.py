"""Counts-GEMM embedding bag (MLP config): C (N x V bf16 counts) @ W (V x E) forward and
C^T @ G backward on hipBLASLt, plain vs split over V (fwd) / N (bwd) into batched GEMMs.

    python tools/bag_gemm_micro.py
"""
import json

import torch


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
    N, V, E, ldc = 4096, 30000, 512, 30016
    C = torch.zeros(N, ldc, device="cuda", dtype=torch.bfloat16)
    C[:, :V] = (torch.rand(N, V, device="cuda") < 0.05).to(torch.bfloat16)
    W = torch.randn(V, E, device="cuda").to(torch.bfloat16)
    G = torch.randn(N, E, device="cuda").to(torch.bfloat16)
    r = {"fwd_plain": ev(lambda: (C[:, :V] @ W).float())}
    ref = (C[:, :V] @ W).float()
    for sk in (4, 8, 16):
        Vk = V // sk
        Cb = C[:, :V].unflatten(1, (sk, Vk)).transpose(0, 1)
        Wb = W.view(sk, Vk, E)
        f = lambda: torch.bmm(Cb, Wb, out_dtype=torch.float32).sum(0)
        r[f"fwd_sk{sk}"] = ev(f)
        r[f"fwd_sk{sk}_err"] = float((f() - ref).abs().max() / ref.abs().max())
    r["bwd_plain"] = ev(lambda: (C[:, :V].t() @ G).float())
    for sk in (2, 4):
        Nk = N // sk
        Cb = C[:, :V].view(sk, Nk, V).transpose(1, 2)
        Gb = G.view(sk, Nk, E)
        r[f"bwd_sk{sk}"] = ev(lambda: torch.bmm(Cb, Gb, out_dtype=torch.float32).sum(0))
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
