#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abj8; mkdir -p $O
for r in 1 2; do
  for L in ab/lib_j16.so ab/lib_j8.so; do
    tag=$(basename $L .so)
    POMS_HIP_LIB=$PWD/$L timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 1 --variants 10 --kinds from_zero --chunks 0,172,129 > $O/kb_${tag}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$tag rc=$rc"; tail -3 $O/kb_${tag}_$r.log; exit $rc; }
    echo "$tag $r: $(grep -o '"chunk": [0-9]*\|"median_us": [0-9.]*' $O/kb_${tag}_$r.log | tr '\n' ' ')"
  done
done
