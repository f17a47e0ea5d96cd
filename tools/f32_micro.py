"""fp32 conv tower forward (conv_pool_f32.hip) at the reference's char page shape: ms and TFLOP/s.

    python tools/f32_micro.py [--N 512] [--L 5000] [--iters 10]
"""
import argparse
import json
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dnn_page_vectors_amd.ops import _common  # noqa: E402
from dnn_page_vectors_amd.ops import conv_pool as cops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=512)
    ap.add_argument("--L", type=int, default=5000)
    ap.add_argument("--V", type=int, default=100)
    ap.add_argument("--E", type=int, default=100)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--bwd", type=int, default=0)
    ap.add_argument("--v2", type=int, default=1, help="role-split forward (0: v1)")
    ap.add_argument("--mask", type=int, default=1, help="dropout keep-bit plane (0: inline hashes)")
    a = ap.parse_args()
    dev = "cuda"
    from dnn_page_vectors_amd.ops._common import lib
    lib().pv_conv_f32_set_v2(a.v2)
    cops.F32_MASK = bool(a.mask)
    torch.manual_seed(0)
    F = 150
    ids = torch.randint(0, a.V, (a.N, a.L), dtype=torch.int32, device=dev)
    table = (torch.randn(a.V, a.E, device=dev) * 0.5).requires_grad_(bool(a.bwd))
    w3 = (torch.randn(F, 3, a.E, device=dev) * 0.1).requires_grad_(bool(a.bwd))
    w4 = (torch.randn(F, 4, a.E, device=dev) * 0.1).requires_grad_(bool(a.bwd))
    b3 = torch.zeros(F, device=dev, requires_grad=bool(a.bwd))
    b4 = torch.zeros(F, device=dev, requires_grad=bool(a.bwd))
    flops = 2.0 * a.N * F * a.E * ((a.L - 2) * 3 + (a.L - 3) * 4)
    for p in (0.25, 0.0):
        def run():
            with _common.precision_scope(types.SimpleNamespace(dtype="fp32")):
                y, _ = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], p, 1, True)
            if a.bwd:
                y.sum().backward()
        run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            run()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.iters
        print(json.dumps({"v2": a.v2, "mask": a.mask, "N": a.N, "L": a.L, "E": a.E, "p": p, "bwd": a.bwd, "ms": round(ms, 3),
                          "fwd_tflops": round(flops / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
