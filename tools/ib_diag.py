"""Localise a disagreement between the loss-kernel generations (loss.hip pv_ib_set_version):
runs the in-batch loss forward + backward with each version on the same inputs and prints
where (row blocks of 256, feature columns) the outputs differ from version 2.

    python tools/ib_diag.py --B 4096 --M 16384 [--clip 0]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dnn_page_vectors_amd.ops import loss as L  # noqa: E402
from dnn_page_vectors_amd.ops._common import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--D", type=int, default=150)
    ap.add_argument("--clip", type=int, default=0)
    ap.add_argument("--vers", default="3,5")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(3)
    q = torch.randn(a.B, a.D, device=dev)
    d = torch.randn(a.M, a.D, device=dev)
    d[: a.B] = q + 0.7 * d[: a.B]
    if a.clip:
        q, d = q.abs(), d.abs()
    qn = torch.nn.functional.normalize(q, dim=1).bfloat16().float()
    dn = torch.nn.functional.normalize(d, dim=1).bfloat16().float()
    pos = torch.arange(a.B, device=dev, dtype=torch.int32)
    w = torch.rand(a.B, device=dev)
    res = {}
    for v in [int(x) for x in a.vers.split(",")]:
        assert lib().pv_ib_set_version(v) == 0
        qq = qn.clone().requires_grad_(True)
        dd = dn.clone().requires_grad_(True)
        loss, _ = L.inbatch_loss(qq, dd, pos, 20.0, bool(a.clip))
        (loss * w).sum().backward()
        torch.cuda.synchronize()
        res[v] = (loss.detach(), qq.grad, dd.grad)
    base = res[min(res)]
    for v, (l, gq, gd) in res.items():
        print(f"version {v}: loss max|d| {float((l - base[0]).abs().max()):.3e}")
        for name, x, b in (("dq", gq, base[1]), ("dd", gd, base[2])):
            diff = (x - b).abs()
            rel = float(diff.norm() / b.norm())
            n = x.shape[0]
            blocks = [(i, float(diff[i:i + 256].max())) for i in range(0, n, 256)]
            bad = [(i, e) for i, e in blocks if e > 1e-2 * float(b.abs().max())]
            cols = diff.max(dim=0).values
            print(f"  {name}: rel {rel:.3e}; bad row blocks {len(bad)}/{len(blocks)} first {bad[:6]}; "
                  f"worst cols {torch.topk(cols, 5).indices.tolist()}; nan {int(torch.isnan(x).sum())}")
        ldiff = (l - base[0]).abs()
        badl = [(i, float(ldiff[i:i + 256].max())) for i in range(0, l.numel(), 256) if float(ldiff[i:i + 256].max()) > 1e-3]
        print(f"  loss bad row blocks {badl[:8]}")


if __name__ == "__main__":
    main()
