"""Micro-benchmark of the CDSSM sparse backward (dW, emit, sort, dTable reduce) at the bench
shape, on uniform or Zipf/topic (synthetic-page) token ids, one process, CUDA events.

    python tools/bwd_micro.py [--N 16384] [--L 2000] [--ids zipf|uniform] [--epw 0,256,512,1024]

epw 0 = the 64-entry reduce4 kernel; others = reduce5 with that many entries per wave.  Every
reduce variant's dTable is checked against reduce4's (fp32 atomics: order differs, so allclose).
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
    ap.add_argument("--ids", default="zipf", choices=["zipf", "uniform"])
    ap.add_argument("--epw", default="0,256,512,1024,2048")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    E, F, FW, EP = 100, 150, 150, 104
    if a.ids == "zipf":
        from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, SyntheticSpec
        sp = SyntheticSpec(vocab_size=a.V, query_length=45, document_length=a.L, num_pages=a.N)
        ids = SyntheticPairs(sp, dev, seed=3).pages.contiguous()
    else:
        ids = torch.randint(1, a.V, (a.N, a.L), dtype=torch.int32, device=dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    table = (torch.randn(a.V, E, generator=g) * 0.05).to(dev)
    w3 = (torch.randn(F, 3, E, generator=g) * 0.05).to(dev)
    w4 = (torch.randn(F, 4, E, generator=g) * 0.05).to(dev)
    bias = torch.zeros(2 * F, device=dev)
    tbl16, wpack = cops.table_bf16(table), cops.pack_weights(w3, w4)
    thr, scale = 64, 256.0 / 192.0
    N, L, V = a.N, a.L, a.V
    L_ = lib()
    s = torch.cuda.current_stream().cuda_stream
    pooled = torch.empty(N, 2 * FW, device=dev)
    argmax = torch.empty(N, 2 * FW, dtype=torch.int32, device=dev)
    check(L_.pv_conv_pool_fwd(P(ids), P(tbl16), P(wpack), P(bias), P(pooled), P(argmax), N, L, V, 7, None, 0, thr, 0,
                              scale, 256, s), "fwd")
    gpool = torch.randn(N, 2 * FW, generator=g).to(dev) * 1e-3
    M = N * cops.SLOTS_PER_SAMPLE
    keys = torch.empty(M, dtype=torch.int32, device=dev)
    vals = torch.empty(M, dtype=torch.int32, device=dev)
    rec = torch.empty(N * 2 * FW, 2, dtype=torch.int32, device=dev)
    skeys, svals = torch.empty_like(keys), torch.empty_like(vals)
    end_bit = max(1, int(V).bit_length())
    tb = int(L_.pv_sort_pairs_temp_bytes(M, end_bit))
    temp = torch.empty(max(tb, 1), dtype=torch.uint8, device=dev)
    wrow = torch.zeros(2 * FW, 4, EP, dtype=torch.bfloat16, device=dev)
    wrow[:FW, :3, :E] = w3
    wrow[FW:, :, :E] = w4
    dw3, dw4, db = torch.zeros_like(w3), torch.zeros_like(w4), torch.zeros(2 * FW, device=dev)

    def emit():
        check(L_.pv_conv_pool_bwd_emit3(P(gpool), P(pooled), P(argmax), P(ids), P(keys), P(vals), P(rec), N, L, V,
                                        scale, s), "emit")

    def sort():
        check(L_.pv_sort_pairs_u32(P(temp), tb, P(keys), P(skeys), P(vals), P(svals), M, end_bit, s), "sort")

    tbi = int(L_.pv_sort_iota_temp_bytes(M, end_bit))
    tempi = torch.empty(max(tbi, 1), dtype=torch.uint8, device=dev)
    svals2 = torch.empty_like(vals)

    def emit_novals():
        check(L_.pv_conv_pool_bwd_emit3(P(gpool), P(pooled), P(argmax), P(ids), P(keys), None, P(rec), N, L, V,
                                        scale, s), "emit")

    def sort_iota():
        check(L_.pv_sort_iota_u32(P(tempi), tbi, P(keys), P(skeys), P(svals2), M, end_bit, s), "sort_iota")

    keys16 = torch.empty(M, dtype=torch.int16, device=dev)
    skeys16 = torch.empty_like(keys16)
    svals3 = torch.empty_like(vals)
    tb16 = int(L_.pv_sort_iota_u16_temp_bytes(M, end_bit))
    temp16 = torch.empty(max(tb16, 1), dtype=torch.uint8, device=dev)

    def emit16():
        check(L_.pv_conv_pool_bwd_emit3_u16(P(gpool), P(pooled), P(argmax), P(ids), P(keys16), P(rec), N, L, V,
                                            scale, s), "emit16")

    def sort16():
        check(L_.pv_sort_iota_u16(P(temp16), tb16, P(keys16), P(skeys16), P(svals3), M, end_bit, s), "sort16")

    def reduce16(out):
        check(L_.pv_conv_pool_bwd_reduce5_u16(P(skeys16), P(svals3), P(rec), P(wrow), P(out), M, 512, L, E, V, 7,
                                              None, 0, thr, 0, s), "reduce16")

    def dw():
        check(L_.pv_conv_pool_bwd_dw(P(gpool), P(pooled), P(argmax), P(ids), P(tbl16), P(dw3), P(dw4), P(db), N, L, E,
                                     V, 7, None, 0, thr, 0, scale, s), "dw")

    def reduce(epw, out):
        if epw == 0:
            check(L_.pv_conv_pool_bwd_reduce4(P(skeys), P(svals), P(rec), P(wrow), P(out), M, L, E, V, 7, None, 0,
                                              thr, 0, s), "reduce4")
        else:
            check(L_.pv_conv_pool_bwd_reduce5(P(skeys), P(svals), P(rec), P(wrow), P(out), M, epw, L, E, V, 7, None,
                                              0, thr, 0, s), "reduce5")

    emit()
    sort()
    sort_iota()
    torch.cuda.synchronize()
    emit16()
    sort16()
    torch.cuda.synchronize()
    print(json.dumps({"sort_iota_vals_equal": bool(torch.equal(svals, svals2)),
                      "sort_u16_vals_equal": bool(torch.equal(svals, svals3))}), flush=True)
    epws = [int(x) for x in a.epw.split(",")]
    ref = torch.zeros(V, E, device=dev)
    reduce(0, ref)
    torch.cuda.synchronize()
    live = int((skeys < V).sum())
    for epw in epws:
        out = torch.zeros(V, E, device=dev)
        reduce(epw, out)
        err = float((out - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
        print(json.dumps({"epw": epw, "rel_err_vs_reduce4": err}), flush=True)
    out16 = torch.zeros(V, E, device=dev)
    reduce16(out16)
    torch.cuda.synchronize()
    print(json.dumps({"reduce_u16_rel_err_vs_reduce4":
                      float((out16 - ref).abs().max() / ref.abs().max().clamp_min(1e-30))}), flush=True)
    res = {k: [] for k in ["emit", "emit_novals", "emit_u16", "sort", "sort_iota", "sort_u16", "dw", "reduce_u16"] +
           [f"reduce_epw{e}" for e in epws]}
    scratch = torch.zeros(V, E, device=dev)
    for _ in range(a.rounds):
        res["emit"].append(ev_time(emit, a.iters))
        res["sort"].append(ev_time(sort, a.iters))
        res["emit_novals"].append(ev_time(emit_novals, a.iters))
        res["sort_iota"].append(ev_time(sort_iota, a.iters))
        res["emit_u16"].append(ev_time(emit16, a.iters))
        res["sort_u16"].append(ev_time(sort16, a.iters))
        res["reduce_u16"].append(ev_time(lambda: reduce16(scratch), a.iters))
        res["dw"].append(ev_time(dw, a.iters))
        for epw in epws:
            res[f"reduce_epw{epw}"].append(ev_time(lambda: reduce(epw, scratch), a.iters))
    out = {k: round(statistics.median(v), 4) for k, v in res.items()}
    out.update({"ids": a.ids, "N": N, "L": L, "entries": M, "live_entries": live})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
