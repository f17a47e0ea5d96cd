"""Same-process A/B of the page-tower dTable reduce: reduce5 vs reduce6 (RB rounds of
weight-row gathers in flight per wave), bench shape, Zipf synthetic pages.

    python tools/reduce_ab.py [--N 16384] [--L 2000] [--rb 2,4,8,16] [--rounds 5]

Every variant's dTable is compared with reduce5's (fp32 atomics between waves: allclose).
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
    ap.add_argument("--rb", default="2,4,8,16")
    ap.add_argument("--epw", type=int, default=512)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, SyntheticSpec
    sp = SyntheticSpec(vocab_size=a.V, query_length=45, document_length=a.L, num_pages=a.N)
    ids = SyntheticPairs(sp, dev, seed=3).pages.contiguous()
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
    check(L_.pv_conv_pool_bwd_emit3_u16(P(gpool), P(pooled), P(argmax), P(ids), P(keys), P(rec), N, L, V, scale, s),
          "emit")
    cops.sort_pairs_iota(keys, skeys, svals, max(1, int(V).bit_length()))
    wrow = cops._weight_rows(w3, w4, cops.EP)

    def r5(out):
        check(L_.pv_conv_pool_bwd_reduce5_u16(P(skeys), P(svals), P(rec), P(wrow), P(out), M, a.epw, L, E, V, 7,
                                              None, 0, thr, 0, s), "reduce5")

    def r6(out, rb):
        check(L_.pv_conv_pool_bwd_reduce6_u16(P(skeys), P(svals), P(rec), P(wrow), P(out), M, a.epw, L, E, V, 7,
                                              None, 0, thr, 0, rb, s), "reduce6")

    def r7(out):
        check(L_.pv_conv_pool_bwd_reduce7_u16(P(skeys), P(svals), P(rec), P(wrow), P(out), M, a.epw, L, E, V, 7,
                                              None, 0, thr, 0, s), "reduce7")

    dw3, dw4, db = torch.zeros_like(w3), torch.zeros_like(w4), torch.zeros(2 * F, device=dev)

    def dw():
        check(L_.pv_conv_pool_bwd_dw(P(gpool), P(pooled), P(argmax), P(ids), P(tbl16), P(dw3), P(dw4), P(db), N, L, E,
                                     V, 7, None, 0, thr, 0, scale, s), "dw")

    ref = torch.zeros(V, E, device=dev)
    r5(ref)
    torch.cuda.synchronize()
    out7 = torch.zeros(V, E, device=dev)
    r7(out7)
    torch.cuda.synchronize()
    err7 = float((out7 - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
    print(json.dumps({"reduce7_rel_err_vs_reduce5": err7}), flush=True)
    assert err7 < 1e-5, err7
    rbs = [int(x) for x in a.rb.split(",") if x]
    for rb in rbs:
        out = torch.zeros(V, E, device=dev)
        r6(out, rb)
        torch.cuda.synchronize()
        err = float((out - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
        print(json.dumps({"rb": rb, "rel_err_vs_reduce5": err}), flush=True)
        assert err < 1e-5, err
    scratch = torch.zeros(V, E, device=dev)
    has_occ = hasattr(L_, "pv_conv_r7_set_occ")
    if has_occ:  # reduce7 capped at 64 VGPRs (8 waves / SIMD, default) vs the compiler's 74 (6 waves)
        L_.pv_conv_r7_set_occ(1)
        L_.pv_conv_r7_set_occ(8)
        out8 = torch.zeros(V, E, device=dev)
        r7(out8)
        L_.pv_conv_r7_set_occ(1)
        torch.cuda.synchronize()
        err8 = float((out8 - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
        print(json.dumps({"reduce7_occ8_rel_err_vs_reduce5": err8}), flush=True)
        assert err8 < 1e-5, err8
    res = {"reduce5": [], "reduce7": [], "reduce7_occ8": [], "dw": []}
    res.update({f"reduce6_rb{rb}": [] for rb in rbs})
    for _ in range(a.rounds):
        res["reduce5"].append(ev_time(lambda: r5(scratch), a.iters))
        res["reduce7"].append(ev_time(lambda: r7(scratch), a.iters))
        if has_occ:
            L_.pv_conv_r7_set_occ(8)
            res["reduce7_occ8"].append(ev_time(lambda: r7(scratch), a.iters))
            L_.pv_conv_r7_set_occ(1)
        res["dw"].append(ev_time(dw, a.iters))
        for rb in rbs:
            res[f"reduce6_rb{rb}"].append(ev_time(lambda: r6(scratch, rb), a.iters))
    out = {k: round(statistics.median(v), 4) for k, v in res.items() if v}
    out.update({"N": N, "L": L, "entries": M, "epw": a.epw})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
