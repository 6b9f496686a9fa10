#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abf; mkdir -p $O
for r in 1 2 3; do
  for f in 0 1; do
    POMS_ALPHA_FOLD=$f timeout -k 10 300 python -u bench.py --ndim 2 --no-cpu-baseline > $O/b2d_f${f}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
    echo "fold=$f r=$r $(tail -1 $O/b2d_f${f}_$r.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
