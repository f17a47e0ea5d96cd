"""Per-kernel totals from a rocprofv3 SQLite (rocpd) result:  python tools/rocpd_stats.py run_results.db [steps]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    c = sqlite3.connect(db)
    q = ("select s.display_name, count(*), sum(d.end - d.start) / 1e3 from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.display_name order by 3 desc")
    rows = list(c.execute(q))
    tot = sum(r[2] for r in rows)
    print("| us / step | calls / step | % | kernel |\n|---:|---:|---:|---|")
    for name, cnt, us in rows[:25]:
        print(f"| {us / steps:.1f} | {cnt / steps:.1f} | {100 * us / tot:.1f} | `{name[:100]}` |")
    print(f"\nTotal GPU kernel time per step: {tot / steps / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
