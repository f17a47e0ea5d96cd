"""Same-process A/B of the whole CDSSM table-gradient chain at the bench shape:

  sorted : emit -> 2-pass LSD radix sort (15-bit keys) -> reduce7 (sorted runs)
  bucket : emit (dead = 0xFFFF) -> ONE radix pass into 128-row buckets -> reduce8 (LDS
           accumulation per bucket item of <= seg entries)

    python tools/table_chain_ab.py [--N 16384] [--L 2000] [--seg 4096,16384,65536] [--rounds 5]

Synthetic Zipf/topic pages (data/synthetic.py) through the real forward (argmax windows,
dropout p = 0.25); reduce8's dTable is compared with reduce7's (fp32 atomics: allclose).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dnn_page_vectors_amd.ops import conv_pool as cops  # noqa: E402
from dnn_page_vectors_amd.ops._common import P, check, lib  # noqa: E402


def ev_time(fn, iters):
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
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--L", type=int, default=2000)
    ap.add_argument("--V", type=int, default=30000)
    ap.add_argument("--seg", default="4096,16384,65536")
    ap.add_argument("--grid", type=int, default=0, help="reduce8 workgroups (0: 2 per CU)")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--uniform", action="store_true", help="uniform token ids instead of Zipf/topic pages")
    a = ap.parse_args()
    dev = torch.device("cuda")
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, SyntheticSpec
    sp = SyntheticSpec(vocab_size=a.V, query_length=45, document_length=a.L, num_pages=a.N)
    ids = SyntheticPairs(sp, dev, seed=3).pages.contiguous()
    if a.uniform:
        ids = torch.randint(1, a.V, ids.shape, dtype=torch.int32, device=dev)
    N, L, V, E, F = a.N, a.L, a.V, 100, 150
    g = torch.Generator(device="cpu").manual_seed(0)
    table = (torch.randn(V, E, generator=g) * 0.05).to(dev)
    w3 = (torch.randn(F, 3, E, generator=g) * 0.05).to(dev)
    w4 = (torch.randn(F, 4, E, generator=g) * 0.05).to(dev)
    bias = torch.zeros(2 * F, device=dev)
    tbl16, wpack = cops.table_bf16(table), cops.pack_weights(w3, w4)
    thr, scale = 64, 256.0 / 192.0
    L_ = lib()
    s = torch.cuda.current_stream().cuda_stream
    pooled = torch.empty(N, 2 * F, device=dev)
    argmax = torch.empty(N, 2 * F, dtype=torch.int32, device=dev)
    check(L_.pv_conv_pool_fwd(P(ids), P(tbl16), P(wpack), P(bias), P(pooled), P(argmax), N, L, V, 7, None, 0, thr, 0,
                              scale, 256, s), "fwd")
    gpool = torch.randn(N, 2 * F, generator=g).to(dev) * 1e-3
    M = N * cops.SLOTS_PER_SAMPLE
    keys = torch.empty(M, dtype=torch.int16, device=dev)
    skeys = torch.empty_like(keys)
    svals = torch.empty(M, dtype=torch.int32, device=dev)
    rec = torch.empty(N * 2 * F, 2, dtype=torch.int32, device=dev)
    wrow = cops._weight_rows(w3, w4, cops.EP)
    totals = torch.empty(256, dtype=torch.int32, device=dev)
    tb = int(L_.pv_rsort_bucket_temp_bytes(M))
    btemp = torch.empty(max(tb, 1), dtype=torch.uint8, device=dev)
    grid = a.grid or 2 * torch.cuda.get_device_properties(dev).multi_processor_count
    out7 = torch.zeros(V, E, device=dev)
    out8 = torch.zeros(V, E, device=dev)

    def emit7():
        check(L_.pv_conv_pool_bwd_emit3_u16(P(gpool), P(pooled), P(argmax), P(ids), P(keys), P(rec), N, L, V, scale,
                                            s), "emit")

    def sort7():
        cops.sort_pairs_iota(keys, skeys, svals, max(1, int(V).bit_length()))

    def red7():
        check(L_.pv_conv_pool_bwd_reduce7_u16(P(skeys), P(svals), P(rec), P(wrow), P(out7), M, 512, L, E, V, 7,
                                              None, 0, thr, 0, s), "reduce7")

    def emit8():
        check(L_.pv_conv_pool_bwd_emit3_u16d(P(gpool), P(pooled), P(argmax), P(ids), P(keys), P(rec), N, L, V, scale,
                                             0xFFFF, s), "emit8")

    def bucket8():
        check(L_.pv_rsort_bucket_u16(P(btemp), tb, P(keys), P(skeys), P(svals), P(totals), M, 7, 8, s), "bucket")

    def red8(seg):
        check(L_.pv_conv_pool_bwd_reduce8(P(skeys), P(svals), P(totals), P(rec), P(wrow), P(out8), seg, grid, L, E,
                                          V, 7, None, 0, thr, 0, s), "reduce8")

    emit7(), sort7(), red7()
    torch.cuda.synchronize()
    live = int(((keys.to(torch.int32) & 0xFFFF) < V).sum())
    segs = [int(x) for x in a.seg.split(",") if x]
    for seg in segs:
        out8.zero_()
        emit8(), bucket8(), red8(seg)
        torch.cuda.synchronize()
        err = float((out8 - out7).abs().max() / out7.abs().max().clamp_min(1e-30))
        print(json.dumps({"seg": seg, "rel_err_vs_reduce7": err, "live_entries": live,
                          "bucket_max": int(totals[:255].max()), "bucket_mean": float(totals[:235].float().mean())}),
              flush=True)
        assert err < 1e-4, err
    res = {"emit": [], "sort2": [], "reduce7": [], "chain7": [], "emit8": [], "bucket1": []}
    res.update({f"reduce8_seg{seg}": [] for seg in segs})
    res.update({f"chain8_seg{seg}": [] for seg in segs})
    for _ in range(a.rounds):
        res["emit"].append(ev_time(emit7, a.iters))
        res["sort2"].append(ev_time(sort7, a.iters))
        res["reduce7"].append(ev_time(red7, a.iters))
        res["chain7"].append(ev_time(lambda: (emit7(), sort7(), red7()), a.iters))
        res["emit8"].append(ev_time(emit8, a.iters))
        res["bucket1"].append(ev_time(bucket8, a.iters))
        for seg in segs:
            res[f"reduce8_seg{seg}"].append(ev_time(lambda: red8(seg), a.iters))
            res[f"chain8_seg{seg}"].append(ev_time(lambda: (emit8(), bucket8(), red8(seg)), a.iters))
    out = {k: round(statistics.median(v), 4) for k, v in res.items()}
    out.update({"N": N, "L": L, "entries": M, "grid": grid})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
