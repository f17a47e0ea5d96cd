"""MX fp8 GEMM (gemm_mx8.hip) at config 5's two shapes — the bag forward (4096 chunks x 30720
vocabulary . table^T, split-K) and the fp8 weight gradient (30000 x 4096 . dZ^T) — with random
e4m3 operands, CUDA-event timed.   python tools/mx8_micro.py [--iters 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from dnn_page_vectors_amd.ops import fp8 as fops

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for name, M, N, K, ks in (("bag_fwd", 4096, 512, 30720, None), ("bag_wgrad", 30000, 512, 4096, 1),
                              ("square", 8192, 8192, 8192, 1)):
        A = (torch.randn(M, K, device=dev, generator=g) * 40).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
        B = (torch.randn(N, K, device=dev, generator=g) * 40).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
        fn = lambda: fops.gemm_mx8(A, B, 1.0, ksplit=ks)  # noqa: E731
        from dnn_page_vectors_amd.ops._common import lib
        r = {"ksplit": ks if ks else fops.mx8_ksplit(M, N, K)}
        for rnd in range(2):
            for ns in (2, 3):  # staging buffers (pv_gemm_mx8_set_stages)
                lib().pv_gemm_mx8_set_stages(ns)
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / a.iters * 1000
                r[f"ns{ns}_us_r{rnd}"] = round(us, 1)
                r[f"ns{ns}_tflops_r{rnd}"] = round(2.0 * M * N * K / us / 1e6, 1)
        lib().pv_gemm_mx8_set_stages(2)
        res[name] = r
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
