#!/bin/bash
# Round 6: A/B of two p = 3 v5 libraries (parity, interleaved kernel times, HBM traffic).
# Usage: tools/r06/ab_trim.sh liba.so libb.so
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab6
mkdir -p $O
A=$1; B=$2
POMS_HIP_LIB=$PWD/$B timeout -k 10 400 python -u -m pytest tests/test_gpu_v5_tiles.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_b.log 2>&1
rc=$?; echo "pytest B rc=$rc"; tail -3 $O/pt_b.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for L in $A $B; do
  tag=$(basename $L .so)
  POMS_HIP_LIB=$PWD/$L timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 2 --variants 10 --kinds apply,jacobi,apply_dot,from_zero >> $O/kb_$tag.log 2>&1
  rc=$?; echo "$tag kb rc=$rc"; tail -4 $O/kb_$tag.log | cut -c1-160
  [ $rc -eq 0 ] || exit $rc
done
done
for L in $A $B; do
  tag=$(basename $L .so)
  for k in apply jacobi; do
    POMS_HIP_LIB=$PWD/$L bash tools/pmc_traffic.sh ${tag}_$k kron_v5 --cells 512 --p 3 --variants 10 --kinds $k > $O/pmc_${tag}_$k.log 2>&1
    rc=$?; echo "$tag $k pmc rc=$rc"; tail -2 $O/pmc_${tag}_$k.log | cut -c1-300
    [ $rc -eq 0 ] || exit $rc
  done
done
