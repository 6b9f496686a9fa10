#!/bin/bash
# rocprofv3 kernel trace of the loopback proxy (rank 1 of 8) with the boundary launch
# on the communication stream: per-queue kernel totals and a timeline window.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03proxytrace; mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3) > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/trace_cycle.py $O/prof/run_kernel_trace.csv 700 > $O/timeline.txt 2>&1; head -16 $O/timeline.txt
