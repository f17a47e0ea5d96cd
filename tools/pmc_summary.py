"""Sum rocprofv3 --pmc counter CSVs per kernel (short names) -> markdown.

    python tools/pmc_summary.py gpurun_out/pmc/p1 gpurun_out/pmc/p2 ... [--match conv_bwd,radix]
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[-70:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    pats = [p for p in a.match.split(",") if p]
    tab = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                if pats and not any(p in r["Kernel_Name"] for p in pats):
                    continue
                tab[k][r["Counter_Name"]] += float(r["Counter_Value"])
                calls[k].add(r.get("Dispatch_Id", ""))
    cols = sorted({c for v in tab.values() for c in v})
    print("| kernel | dispatches | " + " | ".join(cols) + " |")
    print("|---|---:|" + "---:|" * len(cols))
    for k, v in sorted(tab.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        print(f"| `{k}` | {len(calls[k])} | " + " | ".join(f"{v.get(c, 0):.3g}" for c in cols) + " |")


if __name__ == "__main__":
    main()
