"""In-batch / cross-GPU loss kernels: numerics vs the fp32 reference and timing.

    python tools/ib_micro.py [--B 4096] [--M 16384,131072] [--D 150]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dnn_page_vectors_amd.ops import loss as L  # noqa: E402
from dnn_page_vectors_amd.ops import reference as ref  # noqa: E402


def run(qn, dn, pos):
    q = qn.clone().requires_grad_(True)
    d = dn.clone().requires_grad_(True)
    loss, _ = L.inbatch_loss(q, d, pos, 10.0, True)
    loss.sum().backward()
    return loss.detach(), q.grad, d.grad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--M", default="16384,131072")
    ap.add_argument("--D", type=int, default=150)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ib", default="5,3", help="kernel generations to time (loss.hip pv_ib_set_version)")
    ap.add_argument("--glue", default="1", help="ops/loss.py FUSED_GLUE values to time (1 fused finish kernels, "
                                                 "0 the round-5 glue launches)")
    a = ap.parse_args()
    from dnn_page_vectors_amd.ops._common import lib
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for M in [int(x) for x in a.M.split(",")]:
        qn = torch.nn.functional.normalize(torch.randn(a.B, a.D, device=dev, generator=g), dim=1)
        dn = torch.nn.functional.normalize(torch.randn(M, a.D, device=dev, generator=g), dim=1)
        dn[: a.B] = torch.nn.functional.normalize(qn + 0.5 * dn[: a.B], dim=1)  # positives correlated
        qn = qn.bfloat16().float()
        dn = dn.bfloat16().float()
        pos = torch.arange(a.B, device=dev, dtype=torch.int32)  # as the trainer keeps it
        # fp32 oracle
        q = qn.clone().requires_grad_(True)
        d = dn.clone().requires_grad_(True)
        lr, _ = ref.inbatch_softmax_loss(q, d, pos, 10.0, True)
        lr.sum().backward()
        for ver, glue in [(int(v), int(gl)) for v in a.ib.split(",") for gl in a.glue.split(",")]:
            assert lib().pv_ib_set_version(ver) == 0
            L.FUSED_GLUE = bool(glue)
            l, gq, gd = run(qn, dn, pos)
            e = [float((l - lr.detach()).abs().max()), float((gq - q.grad).abs().max() / q.grad.abs().max()),
                 float((gd - d.grad).abs().max() / d.grad.abs().max())]
            ts = []
            for it in range(a.iters + 2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(qn, dn, pos)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            t = sorted(ts[2:])[len(ts[2:]) // 2]
            # GPU time of the same fwd + bwd back to back (CUDA events, no host sync between
            # iterations: the launch latency overlaps as it does inside a training step; the
            # leaves are built once, their .grad reset to None)
            # (own leaves: q / d keep the fp32 oracle's gradients for the next generation's errors)
            qt = qn.clone().requires_grad_(True)
            dt = dn.clone().requires_grad_(True)

            def step():
                qt.grad = None
                dt.grad = None
                loss, _ = L.inbatch_loss(qt, dt, pos, 10.0, True)
                loss.sum().backward()

            step()
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            for _ in range(a.iters):
                step()
            ev1.record()
            torch.cuda.synchronize()
            tg = ev0.elapsed_time(ev1) / a.iters / 1e3
            fl = 2.0 * a.B * M * 160 * 5
            print(f"ib{ver}{'' if glue else ' (round-5 glue)'} M={M}: fwd+bwd {t*1e3:.3f} ms host-synced per call incl. clones ({fl / t / 1e12:.0f} TF/s), "
                  f"{tg*1e3:.3f} ms GPU back to back ({fl / tg / 1e12:.0f} TF/s); "
                  f"err loss {e[0]:.2e} dq {e[1]:.2e} dd {e[2]:.2e}", flush=True)


if __name__ == "__main__":
    main()
