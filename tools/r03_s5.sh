#!/bin/bash
# Split operator call with its reductions on the communication stream: distributed /
# solver parity, the loopback proxy (rank 1 of 8) and its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03s5; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 900 python -u -m pytest tests/test_dist.py tests/test_gpu_solvers.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || stop pytest $rc
for rnd in 1 2; do
  timeout -k 10 300 python tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 5 > $O/proxy_r$rnd.log 2>&1; rc=$?; [ $rc -eq 0 ] || stop proxy $rc
  echo "proxy r$rnd $(grep -o '"ms_per_cycle": [0-9.]*' $O/proxy_r$rnd.log)"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3) > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || stop rocprof $rc
python3 tools/trace_cycle.py $O/prof/run_kernel_trace.csv 700 > $O/timeline.txt 2>&1; sed -n 1,1p $O/timeline.txt; sed -n 14,22p $O/timeline.txt
