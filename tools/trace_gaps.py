"""GPU idle time per training step from a rocprofv3 kernel trace.

    python tools/trace_gaps.py gpurun_out/x/..._kernel_trace.csv [--marker conv_pool_fwd4] [--top 8]

A step starts at each launch of the marker kernel whose duration is above the median of
that kernel's launches (the page tower's conv forward, not the query tower's).  Per step
it prints the span, the union of kernel intervals over all streams (busy), the idle time
(span - busy) and the largest idle gaps with the kernels on both sides: idle between
kernels in an eager step is host-side launch latency the GPU waited for.
"""
import argparse
import csv
import re
import statistics


def short(name: str, n: int = 60) -> str:
    name = re.sub(r"\s+", " ", name)
    name = re.sub(r"^void ", "", name)
    return name if len(name) <= n else name[:n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="conv_pool_fwd4")
    ap.add_argument("--top", type=int, default=8)
    ap.add_argument("--skip", type=int, default=2, help="leading steps to ignore (warmup)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    mk = [k for k in ks if a.marker in k[2]]
    if not mk:
        raise SystemExit(f"no {a.marker} kernels in trace")
    med = statistics.median(e - s for s, e, _ in mk)
    starts = [s for s, e, _ in mk if e - s >= med]
    tot_idle = tot_span = 0.0
    nsteps = 0
    for i in range(a.skip, len(starts) - 1):
        lo, hi = starts[i], starts[i + 1]
        inside = [k for k in ks if lo <= k[0] < hi]
        busy = 0
        cur_s = cur_e = None
        gaps = []
        prev = None
        for s, e, n in inside:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    gaps.append((s - cur_e, short(prev), short(n)))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            if cur_e == e:
                prev = n
        if cur_e is not None:
            busy += min(cur_e, hi) - cur_s
            if hi > cur_e:
                gaps.append((hi - cur_e, short(prev), "<next step>"))
        span = hi - lo
        tot_idle += span - busy
        tot_span += span
        nsteps += 1
        print(f"step {i}: span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms, "
              f"{len(inside)} kernels")
        for g, p, n in sorted(gaps, reverse=True)[:a.top]:
            print(f"    gap {g / 1e3:8.1f} us  after {p}  before {n}")
    if nsteps:
        print(f"mean over {nsteps} steps: span {tot_span / nsteps / 1e6:.3f} ms, idle {tot_idle / nsteps / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
