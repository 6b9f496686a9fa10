#!/bin/bash
# One box: apply cache policy (variants 10 / 104 / 109) and the two-sweeps-from-zero
# y-store policy (quick builds given as arguments), interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/j0ab; mkdir -p $O
for L in "$@"; do
  tag=$(basename $L .so)
  POMS_HIP_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_v5_tiles.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_$tag.log 2>&1
  rc=$?; echo "$tag pytest rc=$rc"; tail -1 $O/pt_$tag.log
  [ $rc -le 1 ] || exit $rc
done
for r in 1 2; do
  timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 2 --variants 10,104 --kinds apply,dot >> $O/kb_cp.log 2>&1 || exit 1
  for L in "$@"; do
    tag=$(basename $L .so)
    POMS_HIP_LIB=$PWD/$L timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 2 --variants 10 --kinds from_zero >> $O/kb_$tag.log 2>&1 || exit 1
  done
done
for f in $O/kb_*.log; do echo "== $f"; grep -h GBps $f | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['variant'], d['kind'], round(d['median_us'],1), round(d['min_us'],1))"; done
