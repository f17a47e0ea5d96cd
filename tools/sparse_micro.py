"""Micro-benchmark of the row-sparse embedding gradient path (parallel/sparse_rows.py) against
the dense table gradient + LazyAdam, at the reference's word-level vocabulary size
(7,556,273 x 100, dssm_cnn/data_helpers.py:143) with ~1% of the rows touched per step.

Per step, single process (the data-parallel exchange is covered by the gloo tests):
  dense : zero the whole flat gradient, scatter the step's row gradients, sum-of-squares /
          non-finite scan over the whole buffer, lazy Adam over the whole table;
  sparse: zero last step's rows, note the ids, scatter, candidate rows (unique), stats over
          the rows, Adam over the row list.

    python tools/sparse_micro.py [--V 7556273] [--E 100] [--touched 0.01] [--steps 10]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dnn_page_vectors_amd.ops.optim import FlatAdam, FlatParams, grad_sumsq_and_finite  # noqa: E402
from dnn_page_vectors_amd.parallel.sparse_rows import SparseTables  # noqa: E402


class _M(torch.nn.Module):
    def __init__(self, V, E):
        super().__init__()
        self.embedding = torch.nn.Parameter(torch.randn(V, E) * 0.05)
        self.dense = torch.nn.Parameter(torch.randn(150, 300) * 0.05)


def run(sparse: bool, V: int, E: int, touched: float, steps: int, dev):
    torch.manual_seed(0)
    m = _M(V, E).to(dev)
    flat = FlatParams(m.named_parameters())
    sp = SparseTables(flat, ["embedding"]) if sparse else None
    opt = FlatAdam(flat, lazy=["embedding"], sparse=sp)
    n_ids = int(V * touched)
    g = torch.Generator(device=dev).manual_seed(1)
    batches = [torch.randint(0, V, (n_ids,), device=dev, generator=g, dtype=torch.int32) for _ in range(4)]
    vals = torch.randn(n_ids, E, device=dev) * 1e-3
    o, k, _ = flat.offsets["embedding"]
    g2 = flat.grad[o:o + k].view(V, E)

    def step(i):
        ids = batches[i % len(batches)]
        if sp is not None:
            flat.zero_grad(skip=sp.ranges())
            sp.begin_step()
            with torch.enable_grad():
                sp.note(m.embedding, ids)
        else:
            flat.zero_grad()
        g2.index_add_(0, ids.long(), vals)  # the backward's row gradients
        flat.grad[-150 * 300:].normal_()
        stats = sp.grad_stats(flat.grad, grad_sumsq_and_finite) if sp is not None else grad_sumsq_and_finite(flat.grad)
        opt.step(stats[1:2])
        if sp is not None:
            sp.finish_step()

    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(steps):
        step(i)
    e.record()
    torch.cuda.synchronize()
    touched = torch.unique(torch.cat(batches).long())
    # the WHOLE table after the run (the rows no step touched must be unchanged as well) and the
    # list of rows some step touched
    return s.elapsed_time(e) / steps, flat.data[o:o + k].view(V, E).clone(), touched


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--V", type=int, default=7_556_273)
    ap.add_argument("--E", type=int, default=100)
    ap.add_argument("--touched", type=float, default=0.01)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    res, tables = {}, {}
    for sparse in (False, True):
        ms, tab, touched = run(sparse, a.V, a.E, a.touched, a.steps, dev)
        res["sparse" if sparse else "dense_lazy"] = round(ms, 3)
        tables[sparse] = tab
        torch.cuda.empty_cache()
    d, s_ = tables[False], tables[True]
    torch.manual_seed(0)  # run()'s initial table
    init = _M(a.V, a.E).embedding.detach().to(dev) if a.V * a.E <= 2_000_000_000 else None
    print(json.dumps({"V": a.V, "E": a.E, "touched_frac": a.touched, "ms_per_step": res,
                      "speedup": round(res["dense_lazy"] / res["sparse"], 2),
                      # every row of the table, and the touched rows on their own
                      "table_equal": bool(torch.equal(d, s_)),
                      "touched_rows": int(touched.numel()),
                      "touched_rows_equal": bool(torch.equal(d[touched], s_[touched])),
                      "touched_rows_changed": None if init is None else
                      bool((s_[touched] != init[touched]).any(dim=1).all()),
                      "max_abs_diff": float((d - s_).abs().max())}))


if __name__ == "__main__":
    main()
