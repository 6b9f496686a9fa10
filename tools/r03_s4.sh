#!/bin/bash
# Vector kernels at 65536 blocks: kernel / full-size / solver parity, then the 3D bench.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03s4}; mkdir -p $O
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_solvers.py tests/test_gpu_golden.py \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || stop pytest $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-200; [ $rc -eq 0 ] || stop bench $rc
echo "session done"
