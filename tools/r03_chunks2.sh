#!/bin/bash
# Confirmation: two-sweeps-from-zero and Jacobi at the auto chunk (172 planes at 515^3)
# against 6-8 chunks, three interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03chunks2; mkdir -p $O
timeout -k 10 600 python tools/kernel_bench.py --cells 512 --p 3 --reps 20 --rounds 3 --kinds from_zero,jacobi --chunks 0,86,74,65 > $O/kb.log 2>&1; rc=$?
python3 -c "
import json
rows=[json.loads(l) for l in open('$O/kb.log') if l.startswith('{')]
for r in rows: print(r['kind'], r['chunk'], round(r['median_us'],1), round(r['min_us'],1))
"
exit $rc
