#!/bin/bash
# rocprofv3 kernel statistics of a short 3D bench run (2 timed cycles + 1 warm-up).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03prof}; mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline) > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 $O/prof.log | cut -c1-200; exit $rc
