#!/bin/bash
# Speculative smoother: parity (native step-by-step / speculative / Python loop), the
# 2D cycle with and without it (interleaved), the 3D bench unchanged.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r04spec}; mkdir -p $O
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_solvers.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "speculative or native_pcg or damped_jacobi or device_reduction" > $O/pytest_spec.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_spec.log; [ $rc -eq 0 ] || stop pytest $rc
for r in 1 2; do
  for m in 0 1; do
    POMS_PCG_SPEC=$m timeout -k 10 300 python bench.py --ndim 2 --no-cpu-baseline > $O/bench2d_spec${m}_$r.log 2>&1; rc=$?; echo "2d spec=$m rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench2d_spec${m}_$r.log)"; [ $rc -eq 0 ] || stop bench2d $rc
  done
done
echo "session done"
