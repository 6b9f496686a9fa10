#!/usr/bin/env python3
"""Effective clock of each kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace run
(MI355X_MICROARCH.md, DVFS give-back: clock ~= GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time).

    python tools/clock_summary.py gpurun_out/<dir> [kernel-substring ...]
"""
import collections
import csv
import statistics
import sys
from pathlib import Path


def main():
    root = Path(sys.argv[1])
    subs = sys.argv[2:]
    dur = {}
    for f in root.rglob("*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    cnt = collections.defaultdict(dict)
    names = {}
    for f in root.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            d = r["Dispatch_Id"]
            cnt[d][r["Counter_Name"]] = cnt[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[d] = r.get("Kernel_Name", "")
    per = collections.defaultdict(list)
    for d, c in cnt.items():
        if d not in dur or "GRBM_GUI_ACTIVE" not in c or dur[d] < 50e-6:
            continue
        nm = names[d]
        if subs and not any(s in nm for s in subs):
            continue
        per[nm.split("(")[0][-80:]].append((dur[d], c["GRBM_GUI_ACTIVE"] / 8.0 / dur[d] / 1e9))
    for nm, v in per.items():
        ghz = [x[1] for x in v]
        us = [x[0] * 1e6 for x in v]
        print(f"{nm}\n   n={len(v)}  wall median {statistics.median(us):8.1f} us   clock median {statistics.median(ghz):.3f} GHz "
              f"(min {min(ghz):.3f}, max {max(ghz):.3f})")


if __name__ == "__main__":
    main()
