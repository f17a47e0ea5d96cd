"""Dense-layer backward GEMMs (K4): library vs in-tree kernels on the model shapes.

    python tools/dense_bwd_micro.py

dgrad dx = dz W   : torch (hipBLASLt) vs dense.hip linear_act reading W transposed (pv_linear_dgrad)
wgrad dW = dz^T x : ops/dense._wgrad (batched hipBLASLt + column sums) vs the in-tree
                    wgrad kernel (pv_linear_wgrad) where present.
"""
from __future__ import annotations

import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dnn_page_vectors_amd.ops import dense as D  # noqa: E402
from dnn_page_vectors_amd.ops._common import P, lib, stream  # noqa: E402

SHAPES = [  # (rows M, out N, in K): CDSSM dense (page / query tower), MLP tower layers
    (16384, 150, 300), (4096, 150, 300), (16384, 512, 512), (16384, 128, 512), (4096, 512, 512)]


def timeit(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    dev = torch.device("cuda")
    L_ = lib()
    has_wg = hasattr(L_, "pv_linear_wgrad")
    for M, N, K in SHAPES:
        dz = torch.randn(M, N, device=dev)
        w = torch.randn(N, K, device=dev) * 0.05
        x = torch.randn(M, K, device=dev)
        ref_dx = dz @ w
        dx = torch.empty(M, K, device=dev)

        def hip_dgrad():
            L_.pv_linear_dgrad(P(dz), 0, P(w), 0, P(dx), M, N, K, stream(dev))

        hip_dgrad()
        e_dx = float((dx - ref_dx).abs().max() / ref_dx.abs().max())
        t_lib = timeit(lambda: dz @ w)
        t_hip = timeit(hip_dgrad)
        ref_dw = dz.t() @ x
        t_wl = timeit(lambda: D._wgrad(dz, x))
        line = (f"M={M} N={N} K={K}: dgrad lib {t_lib:.1f} us, hip {t_hip:.1f} us, "
                f"err {e_dx:.1e}; wgrad lib {t_wl:.1f} us")
        if has_wg:
            dw = torch.empty(N, K, device=dev)
            D.wgrad_hip(dz, x, out=dw)
            e_dw = float((dw - ref_dw).abs().max() / ref_dw.abs().max())
            t_wh = timeit(lambda: D.wgrad_hip(dz, x, out=dw))
            line += f", hip {t_wh:.1f} us err {e_dw:.1e}"
            for wgt in (256, 512, 1024):
                D._WG_TARGET = wgt
                line += f", wg{wgt} {timeit(lambda: D.wgrad_hip(dz, x, out=dw)):.1f}"
            D._WG_TARGET = 512
            for tl in (64, 128):
                D.wgrad_hip(dz, x, out=dw, tile=tl)
                e_t = float((dw - ref_dw).abs().max() / ref_dw.abs().max())
                line += f", tile{tl} {timeit(lambda: D.wgrad_hip(dz, x, out=dw, tile=tl)):.1f} us err {e_t:.1e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
