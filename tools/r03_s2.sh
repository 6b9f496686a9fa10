#!/bin/bash
# Host-reduced partials: native-pcg parity (bitwise against the Python loop), the 2D
# and 3D benches; then the RCCL channel knobs on the loopback proxy.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03s2}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || stop pytest $rc
timeout -k 10 300 python bench.py --ndim 2 --no-cpu-baseline > $O/bench_2d.log 2>&1; rc=$?; echo "bench2d rc=$rc"; tail -1 $O/bench_2d.log | cut -c1-200; [ $rc -eq 0 ] || stop bench2d $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-200; [ $rc -eq 0 ] || stop bench $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof2d -o run -- python3 $GRAFT_REPO_ROOT/bench.py --ndim 2 --no-cpu-baseline --steps 10) > $O/prof2d.log 2>&1
rc=$?; echo "rocprof2d rc=$rc"; [ $rc -eq 0 ] || stop rocprof2d $rc
bash tools/r03_rccl_knobs.sh ${1:-r03s2}/knobs
