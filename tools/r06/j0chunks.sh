#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/j0c; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 2 --variants 10 --kinds from_zero,jacobi --chunks 0,86,103,129,172 > $O/kb_$r.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
  python3 -c "
import json
for l in open('$O/kb_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['kind'], d['chunk'], round(d['median_us'],1), round(d['min_us'],1))"
done
