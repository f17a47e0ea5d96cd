"""Same-process A/B of the page-tower dTable reduce (conv_bwd_reduce7_kernel) at the bench
shape, Zipf synthetic pages: 2-byte vs 4-byte sort keys, 64-VGPR cap (8 waves / SIMD, the
default) vs the compiler's allocation, and the dW kernel beside it for scale.

    python tools/reduce_ab.py [--N 16384] [--L 2000] [--rounds 5]

Every arm's dTable is compared with the default arm's (fp32 atomics between waves: allclose).
(The reduce4 / 5 / 6 generations this tool once compared are gone: docs/PERF.md.)
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
    check(L_.pv_conv_pool_fwd2(P(ids), P(tbl16), P(wpack), P(bias[:F]), P(bias[F:]), P(pooled), P(argmax), N, L, V, 7,
                               None, 0, thr, 0, scale, 256, s, None, 0), "fwd")
    gpool = torch.randn(N, 2 * F, generator=g).to(dev) * 1e-3
    M = N * cops.SLOTS_PER_SAMPLE
    keys = torch.empty(M, dtype=torch.int16, device=dev)
    skeys = torch.empty_like(keys)
    svals = torch.empty(M, dtype=torch.int32, device=dev)
    rec = torch.empty(N * 2 * F, 2, dtype=torch.int32, device=dev)
    check(L_.pv_conv_pool_bwd_emit3_u16(P(gpool), P(pooled), P(argmax), P(ids), P(keys), P(rec), N, L, V, scale, s),
          "emit")
    end_bit = max(1, int(V).bit_length())
    cops.sort_pairs_iota(keys, skeys, svals, end_bit)
    keys32 = keys.to(torch.int32) & 0xFFFF
    skeys32 = torch.empty_like(keys32)
    svals32 = torch.empty_like(svals)
    cops.sort_pairs_iota(keys32, skeys32, svals32, end_bit)
    wrow = cops._weight_rows(w3, w4, cops.EP)

    def r7(out, k32=False):
        fn = "pv_conv_pool_bwd_reduce7" if k32 else "pv_conv_pool_bwd_reduce7_u16"
        sk, sv = (skeys32, svals32) if k32 else (skeys, svals)
        check(getattr(L_, fn)(P(sk), P(sv), P(rec), P(wrow), P(out), M, a.epw, L, E, V, 7, None, 0, thr, 0, s), fn)

    dw3, dw4, db = torch.zeros_like(w3), torch.zeros_like(w4), torch.zeros(2 * F, device=dev)

    def dw():
        check(L_.pv_conv_pool_bwd_dw2(P(gpool), P(pooled), P(argmax), P(ids), P(tbl16), P(dw3), P(dw4), P(db[:F]),
                                      P(db[F:]), N, L, E, V, 7, None, 0, thr, 0, scale, s), "dw")

    def occ1(fn):
        def run():
            L_.pv_conv_r7_set_occ(1)
            try:
                fn()
            finally:
                L_.pv_conv_r7_set_occ(8)
        return run

    ref = torch.zeros(V, E, device=dev)
    r7(ref)
    arms = {"reduce7_u16": lambda o: r7(o), "reduce7_u32": lambda o: r7(o, True),
            "reduce7_u16_occ1": lambda o: occ1(lambda: r7(o))()}
    for name, fn in arms.items():
        out = torch.zeros(V, E, device=dev)
        fn(out)
        torch.cuda.synchronize()
        err = float((out - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
        print(json.dumps({name + "_rel_err": err}), flush=True)
        assert err < 1e-5, (name, err)
    scratch = torch.zeros(V, E, device=dev)
    res = {k: [] for k in list(arms) + ["dw"]}
    for _ in range(a.rounds):
        for name, fn in arms.items():
            res[name].append(ev_time(lambda: fn(scratch), a.iters))
        res["dw"].append(ev_time(dw, a.iters))
    out = {k: round(statistics.median(v), 4) for k, v in res.items() if v}
    out.update({"N": N, "L": L, "entries": M, "epw": a.epw})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
