"""One training step's kernel timeline from a rocprofv3 kernel trace: start / end (us from the
step's first page-conv launch), duration and queue of every kernel above --min-us.

    python tools/timeline.py gpurun_out/x/..._kernel_trace.csv [--marker conv_pool_fwd7] [--step -3]
"""
import argparse
import csv
import re
import statistics


def short(n: str) -> str:
    n = re.sub(r"^void ", "", n)
    return re.sub(r"\(.*", "", n)[:64]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="conv_pool_fwd7")
    ap.add_argument("--step", type=int, default=-3, help="which step (python index over detected steps)")
    ap.add_argument("--min-us", type=float, default=5.0)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
    mk = [k for k in ks if a.marker in k[2]]
    med = statistics.median(e - s for s, e, *_ in mk)
    starts = [s for s, e, *_ in mk if e - s >= med]
    i = a.step % (len(starts) - 1)
    lo, hi = starts[i], starts[i + 1]
    for s, e, n, q in ks:
        if lo <= s < hi and (e - s) / 1e3 >= a.min_us:
            print(f"{(s - lo) / 1e3:8.1f} {(e - lo) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} {short(n)}")
    print(f"step span {(hi - lo) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
