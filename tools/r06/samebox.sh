#!/bin/bash
# ubench march vs the library's memory-only apply (variant 101) on one box
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/samebox; mkdir -p $O
export POMS_HIP_LIB=$PWD/ab/lib_m1nt.so
for r in 1 2; do
  timeout -k 10 120 tools/r06/ubench_march2.bin 1 > $O/ub_$r.log 2>&1; rc=$?; cat $O/ub_$r.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 1 --variants 101,10 --kinds apply > $O/kb_$r.log 2>&1
  rc=$?; cut -c1-140 $O/kb_$r.log | grep variant; [ $rc -eq 0 ] || exit $rc
done
