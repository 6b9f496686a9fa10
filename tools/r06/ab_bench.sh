#!/bin/bash
# Round 6: interleaved 3D bench (and kernel_bench) of two libraries on one box.
# Usage: tools/r06/ab_bench.sh liba.so libb.so [rounds]
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abb; mkdir -p $O
for r in $(seq 1 ${3:-2}); do
  for L in $1 $2; do
    tag=$(basename $L .so)
    POMS_HIP_LIB=$PWD/$L timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_${tag}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$tag bench rc=$rc"; exit $rc; }
    python3 -c "
import json,sys
d=json.loads([x for x in open('$O/bench_${tag}_$r.log') if x.startswith('{')][-1])
print('$tag', $r, round(d['ms_per_step'],2), round(d['roofline']['avg_launch_us'],1), round(d['kron_spmv']['median_launch_us'],1))"
  done
done
