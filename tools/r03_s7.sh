#!/bin/bash
# Post-smoother iterating in the V-cycle's own xf: solver / golden / dist parity, bench.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03s7; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_golden.py tests/test_dist.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-200
