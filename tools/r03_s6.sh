#!/bin/bash
# J0 with the halved chunk: parity (kernels, full size, solvers, golden, dist) and timings.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03s6; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_solvers.py tests/test_gpu_golden.py tests/test_dist.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 20 --rounds 2 --kinds from_zero --chunks 0,172 2>&1 | grep -v amdgpu.ids | cut -c1-140 | tee $O/kb.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-200
