#!/bin/bash
# Axis-0 chunk sweep of the 515^3 v5 launches (0 = auto_chunk's pick).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03chunks; mkdir -p $O
timeout -k 10 500 python tools/kernel_bench.py --cells 512 --p 3 --reps 15 --rounds 2 --kinds jacobi,apply,from_zero --chunks 0,64,86,103,129,258 > $O/kb.log 2>&1; rc=$?
python3 -c "
import json
rows=[json.loads(l) for l in open('$O/kb.log') if l.startswith('{')]
for r in rows: print(r['kind'], r['chunk'], round(r['median_us'],1), round(r['min_us'],1))
"
exit $rc
