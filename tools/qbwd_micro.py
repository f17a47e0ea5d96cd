"""Query-tower backward A/B: dTable by the per-sample dense dX kernel vs emit -> sort ->
reduce (cops.DENSE_DX), interleaved in one process, Zipf token ids, dropout 0.25.

    python tools/qbwd_micro.py --shapes 4096x45 1024x250
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dnn_page_vectors_amd.ops import conv_pool as cops  # noqa: E402


def ev(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=["4096x45", "1024x250"])
    ap.add_argument("--V", type=int, default=30000)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    cops.DENSE_DX_MAXL = 256
    dev = torch.device("cuda")
    E, F = 100, 150
    g = torch.Generator(device=dev).manual_seed(0)
    ranks = torch.arange(1, a.V, dtype=torch.float32, device=dev)
    probs = ranks.pow(-1.0)
    for shp in a.shapes:
        N, L = (int(x) for x in shp.split("x"))
        ids = (torch.multinomial(probs / probs.sum(), N * L, replacement=True, generator=g) + 1).view(N, L)
        ids = ids.to(torch.int32)
        table = torch.nn.Parameter(torch.randn(a.V, E, device=dev) * 0.05)
        w3 = torch.nn.Parameter(torch.randn(F, 3, E, device=dev) * 0.05)
        w4 = torch.nn.Parameter(torch.randn(F, 4, E, device=dev) * 0.05)
        b3 = torch.nn.Parameter(torch.zeros(F, device=dev))
        b4 = torch.nn.Parameter(torch.zeros(F, device=dev))
        cache = (cops.table_bf16(table.detach()), cops.pack_weights(w3.detach(), w4.detach()))
        gout = torch.randn(N, 2 * F, device=dev) * 1e-3

        def fwd():
            with torch.no_grad():
                cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], 0.25, 7, True, compute_cache=cache)

        def fwd_bwd():
            pooled, _ = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], 0.25, 7, True,
                                                     compute_cache=cache)
            pooled.backward(gout)

        res = {True: [], False: []}
        for _ in range(a.rounds):
            for dense in (False, True):
                cops.DENSE_DX = dense
                res[dense].append(ev(fwd_bwd, a.iters) - ev(fwd, a.iters))
        cops.DENSE_DX = True
        print(json.dumps({"N": N, "L": L, "bwd_ms_sort_path": round(statistics.median(res[False]), 4),
                          "bwd_ms_dense_dx": round(statistics.median(res[True]), 4)}), flush=True)


if __name__ == "__main__":
    main()
