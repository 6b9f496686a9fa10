#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_traffic.py gpurun_out/pmc <kernel-substring> <dof> [out.json [p variant]]

Corrections (MI355X_MICROARCH.md, HBM section, gfx950): FETCH_SIZE counts half
of the bytes of wide streaming reads (x2); WRITE_SIZE is exact for streaming
stores.  Our 8-B-per-lane access pattern was calibrated on the vector dot
kernel (16 algorithmic B/DOF -> 8.2 raw FETCH B/DOF) and on the Jacobi sweep's
stores (8.0 algorithmic B/DOF -> 8.0 WRITE B/DOF).  Both counters are in KiB.
"""
import collections
import csv
import json
import sys
from pathlib import Path


def mean_counter(root: Path, counter: str, substr: str):
    vals = []
    for f in sorted(root.rglob("*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and substr in r.get("Kernel_Name", ""):
                vals.append(float(r["Counter_Value"]))
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    root, substr, dof = Path(sys.argv[1]), sys.argv[2], float(sys.argv[3])
    fetch, nf = mean_counter(root, "FETCH_SIZE", substr)
    write, nw = mean_counter(root, "WRITE_SIZE", substr)
    if fetch is None or write is None:
        raise SystemExit("counters not found")
    rd = 2.0 * fetch * 1024.0
    wr = write * 1024.0
    out = {"kernel_substring": substr, "dispatches": [nf, nw], "fetch_kib_raw": fetch, "write_kib": write,
           "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
           "hbm_bytes_per_launch": rd + wr, "bytes_per_dof": (rd + wr) / dof,
           "correction": "read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE; KiB -> bytes"}
    if len(sys.argv) > 6:   # optional provenance: p, kernel variant (bench.py matches them)
        out["p"], out["variant"] = int(sys.argv[5]), int(sys.argv[6])
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 4:
        Path(sys.argv[4]).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
