#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output: mean counter value per dispatch, per kernel.

    python tools/pmc_summary.py gpurun_out/pmc [filter-substring]
"""
import collections
import csv
import sys
from pathlib import Path


def main():
    root = Path(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(root.rglob("*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if filt and filt not in name:
                continue
            key = (name, r.get("Dispatch_Id", ""))
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in vals.items():
        short = name.split("(")[0][-70:]
        print(short)
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {sum(v) / len(v):16.4g}   (n={len(v)})")


if __name__ == "__main__":
    main()
