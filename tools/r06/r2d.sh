#!/bin/bash
# Round 6: 2D p = 3 v3 tile height (POMS_V3_2D_R rows per wave, 8 waves): sweep and
# apply + dot times at 1024^2, then the 2D bench cycle for each height.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2d; mkdir -p $O
for r in 2 3 4 5 6 2; do
  POMS_V3_2D_R=$r timeout -k 10 120 python tools/kernel_bench.py --ndim 2 --cells 1024 --p 3 --reps 30 --rounds 2 --kinds jacobi,apply_dot > $O/kb_$r.log 2>&1
  rc=$?; echo "R=$r: $(grep -o '"kind": "[a-z_]*", "median_us": [0-9.]*' $O/kb_$r.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
for r in 2 5 4 2 5 4; do
  POMS_V3_2D_R=$r timeout -k 10 300 python bench.py --ndim 2 --no-cpu-baseline > $O/bench_$r.log 2>&1
  rc=$?; echo "bench R=$r: $(tail -1 $O/bench_$r.log | grep -o '"ms_per_step": [0-9.]*')"; [ $rc -eq 0 ] || exit $rc
done
