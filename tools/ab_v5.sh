#!/bin/bash
# A/B of two quick (p = 3) v5 builds: parity of the fast march, kernel timings at
# 515^3, the headline bench.  Usage: tools/ab_v5.sh liba.so libb.so
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab
mkdir -p $O
for L in "$@"; do
  tag=$(basename $L .so)
  POMS_HIP_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_v5_tiles.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pt_$tag.log 2>&1
  rc=$?; echo "$tag pytest rc=$rc"; tail -3 $O/pt_$tag.log
  [ $rc -le 1 ] || exit $rc
done
for L in "$@" "$@"; do
  tag=$(basename $L .so)
  POMS_HIP_LIB=$PWD/$L timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 3 --variants 10 --kinds apply,jacobi,residual >> $O/kb_$tag.log 2>&1
  rc=$?; echo "$tag kb rc=$rc"; tail -3 $O/kb_$tag.log
  [ $rc -eq 0 ] || exit $rc
done
[ -n "${AB_NOBENCH:-}" ] && exit 0
for L in "$@"; do
  tag=$(basename $L .so)
  POMS_HIP_LIB=$PWD/$L timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench_$tag.log 2>&1
  rc=$?; echo "$tag bench rc=$rc"; tail -1 $O/bench_$tag.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
