"""Render a rocprofv3 --kernel-trace --stats CSV (or its rocpd SQLite .db) into a markdown table.

    python tools/prof_summary.py gpurun_out/prof_all/cdssm/cdssm_kernel_stats.csv --steps 13 \
        --title "..." --cmd "..." > profiles/x.md
"""
import argparse
import csv
import re


def short(name: str, n: int = 110) -> str:
    name = re.sub(r"\s+", " ", name)
    return name if len(name) <= n else name[:n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=float, required=True, help="dispatched steps (warmup + timed)")
    ap.add_argument("--title", default="kernel stats")
    ap.add_argument("--cmd", default="")
    ap.add_argument("--note", default="")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    if a.csv.endswith(".db"):  # rocprofv3's default rocpd (SQLite) output: the top_kernels view (us)
        import sqlite3

        con = sqlite3.connect(a.csv)
        rows = [{"Name": n, "Calls": c, "TotalDurationNs": t * 1e3, "Percentage": p}
                for n, c, t, _, p in con.execute("select * from top_kernels order by total_duration desc")]
    else:
        rows = list(csv.DictReader(open(a.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {a.title}\n")
    if a.cmd:
        print(f"Command: `{a.cmd}`\n")
    if a.note:
        print(a.note + "\n")
    print("| us / step | calls / step | % | kernel |")
    print("|---:|---:|---:|---|")
    for r in rows[:a.top]:
        print(f"| {float(r['TotalDurationNs']) / a.steps / 1e3:.1f} | {int(r['Calls']) / a.steps:.1f} | "
              f"{float(r['Percentage']):.1f} | `{short(r['Name'])}` |")
    print(f"\nTotal GPU kernel time per step: {tot / a.steps / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
