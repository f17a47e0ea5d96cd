"""dTable sort micro-benchmark: the in-tree LSD radix sort (radix_sort.hip) at its automatic
items-per-thread and forced ones, same process, interleaved, at the conv-backward shapes
(2-byte keys < 2^15, values = positions).  (The rocPRIM onesweep and counting-sort arms it
once compared are gone: docs/PERF.md "dTable sort".)

    python tools/sort_micro.py --M 17203200 4300800
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dnn_page_vectors_amd.ops import conv_pool as cops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="*", default=[17_203_200, 4_300_800])
    ap.add_argument("--end-bit", type=int, default=15)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--ipt", type=int, nargs="*", default=[4, 16, 32], help="forced items-per-thread arms")
    a = ap.parse_args()
    dev = torch.device("cuda")
    for M in a.M:
        # Zipf-like token keys with a dead-entry sentinel, as the emit kernel writes them
        r = torch.rand(M, device=dev)
        keys = (r ** 4 * 29999).to(torch.int16)
        keys[::5] = 30000
        skeys = torch.empty_like(keys)
        svals = torch.empty(M, dtype=torch.int32, device=dev)
        res = {}
        lib = cops.lib()
        ref_k = ref_v = None
        arms = ["rsort"] + [f"rsort_ipt{i}" for i in a.ipt]

        def run(arm):
            if arm.startswith("rsort_ipt"):
                lib.pv_rsort_set_ipt(int(arm[9:]))
                try:
                    cops.sort_pairs_iota(keys, skeys, svals, a.end_bit)
                finally:
                    lib.pv_rsort_set_ipt(0)
            else:
                cops.sort_pairs_iota(keys, skeys, svals, a.end_bit)

        for arm in arms:
            run(arm)  # warm + every arm must give the same (stable) result
            torch.cuda.synchronize()
            if ref_k is None:
                ref_k, ref_v = skeys.clone(), svals.clone()
            else:
                assert torch.equal(skeys, ref_k) and torch.equal(svals, ref_v), arm
        times = {arm: [] for arm in arms}
        for _ in range(a.iters):
            for arm in arms:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(arm)
                e1.record()
                e1.synchronize()
                times[arm].append(e0.elapsed_time(e1))
        for impl, t in times.items():
            t.sort()
            res[impl + "_ms_median"] = round(t[len(t) // 2], 4)
        print(json.dumps({"M": M, **res}), flush=True)


if __name__ == "__main__":
    main()
