"""BERT FFN forward + backward at the config-4 token count: hipBLASLt fused epilogues
(lt_gemm.hip, PAGEVEC_FFN_LT=1) vs plain GEMMs + bias_gelu kernels, CUDA-event timed in one
process.   python tools/ffn_micro.py [--T 73728] [--H 768] [--I 3072]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=73728)
    ap.add_argument("--H", type=int, default=768)
    ap.add_argument("--I", type=int, default=3072)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from dnn_page_vectors_amd.ops import transformer as tops

    dev = torch.device("cuda")
    x = torch.randn(a.T, a.H, device=dev).bfloat16().requires_grad_(True)
    w1 = (torch.randn(a.I, a.H, device=dev) / a.H ** 0.5).requires_grad_(True)
    b1 = torch.zeros(a.I, device=dev, requires_grad=True)
    w2 = (torch.randn(a.H, a.I, device=dev) / a.I ** 0.5).requires_grad_(True)
    gy = torch.randn(a.T, a.H, device=dev).bfloat16()
    r = {"shape": [a.T, a.H, a.I]}
    arms = {"plain": (0, 0, 0), "lt": (1, 0, 0), "lt_lin": (1, 1, 0), "lt_lin_tune": (1, 1, 1)}
    for rnd in range(2):
        for arm, (ffn, lin, tune) in arms.items():
            tops.FFN_LT, tops.LINEAR_LT, tops.LT_TUNE = bool(ffn), bool(lin), bool(tune)

            def step():
                y = tops.ffn(x, w1, b1, w2)
                y.backward(gy)
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                step()
            e1.record()
            torch.cuda.synchronize()
            r[f"{arm}_ms_r{rnd}"] = round(e0.elapsed_time(e1) / a.iters, 4)
    r["lt_ok"] = {str(k): v for k, v in tops._LT_OK.items()}
    flops = 3 * 2 * 2.0 * a.T * a.H * a.I
    for arm in arms:
        r[f"{arm}_tflops"] = round(flops / min(r[f"{arm}_ms_r0"], r[f"{arm}_ms_r1"]) / 1e9, 1)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
