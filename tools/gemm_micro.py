"""hipBLASLt timing of the BERT-base linear-layer GEMMs (fwd / dgrad / wgrad) and of wgrad
alternatives (bf16 out, split-K over tokens with fp32 partial sums).

    python tools/gemm_micro.py [--tokens 65536 8192]
"""
import argparse
import json

import torch


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, nargs="+", default=[65536, 8192])
    a = ap.parse_args()
    dev = "cuda"
    a_ = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    b_ = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: a_ @ b_, iters=10)
    print(json.dumps({"square_8192": f"{t:.3f} ms {2 * 8192 ** 3 / t / 1e9:.0f} TF/s"}), flush=True)
    shapes = [(768, 2304), (768, 768), (768, 3072), (3072, 768)]
    for T in a.tokens:
        for K, N in shapes:
            x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
            b = torch.randn(N, device=dev, dtype=torch.bfloat16)
            dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
            fl = 2.0 * T * K * N
            r = {"T": T, "K": K, "N": N}
            r["fwd"] = timeit(lambda: torch.addmm(b, x, w.t()))
            r["dgrad"] = timeit(lambda: dy @ w)
            r["wgrad_f32"] = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
            r["wgrad_bf16"] = timeit(lambda: (dy.t() @ x))
            r["wgrad_xT_dy_f32"] = timeit(lambda: torch.mm(x.t(), dy, out_dtype=torch.float32))
            for sk in (4, 8, 16):
                if T % sk:
                    continue
                dy3 = dy.view(sk, T // sk, N)
                x3 = x.view(sk, T // sk, K)
                try:
                    r[f"wgrad_sk{sk}_f32"] = timeit(
                        lambda: torch.bmm(dy3.transpose(1, 2), x3, out_dtype=torch.float32).sum(0))
                except Exception as ex:  # bmm.dtype missing
                    r[f"wgrad_sk{sk}_f32"] = str(ex)[:60]
                r[f"wgrad_sk{sk}_bf16"] = timeit(lambda: torch.bmm(dy3.transpose(1, 2), x3).sum(0, dtype=torch.float32))
            for k, v in list(r.items()):
                if isinstance(v, float) and k not in ("T", "K", "N"):
                    r[k] = f"{v:.3f} ms {fl / v / 1e9:.0f} TF/s"
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
