#!/bin/bash
# A/B of two library builds on one box through POMS_HIP_LIB (interleaved): GPU solver
# parity with the new build first, then 2D and 3D V-cycles.  Usage: r03_ab_lib.sh OUT OLD.so NEW.so
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03ablib}; OLD=$2; NEW=$3; mkdir -p $O
POMS_HIP_LIB=$PWD/$NEW timeout -k 10 600 python -u -m pytest tests/test_gpu_solvers.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then L=$OLD; else L=$NEW; fi
    POMS_HIP_LIB=$PWD/$L timeout -k 10 200 python bench.py --ndim 2 --no-cpu-baseline --steps 40 > $O/b2d_${v}_r$rep.log 2>&1 || exit 1
    echo "2D $v rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $O/b2d_${v}_r$rep.log)"
  done
done
for v in old new; do
  if [ $v = old ]; then L=$OLD; else L=$NEW; fi
  POMS_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > $O/b3d_${v}.log 2>&1 || exit 1
  echo "3D $v $(grep -o '"ms_per_step": [0-9.]*' $O/b3d_${v}.log)"
done
