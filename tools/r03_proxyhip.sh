#!/bin/bash
# HIP API trace (host side) + kernel trace of the loopback proxy, rank 1 of 8.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03proxyhip; mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 2) > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; ls $O/prof; exit $rc
