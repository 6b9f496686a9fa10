#!/bin/bash
# In-process A/B of the 2D cycle (speculative / graph modes) and a kernel trace of
# the loopback proxy (rank 1 of 8) for its timeline.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
O=gpurun_out/${1:-r04ab}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 300 python tools/cycle_ab.py --ndim 2 --cells 1024 --modes "POMS_PCG_SPEC=0,POMS_PCG_GRAPH=0;POMS_PCG_SPEC=1,POMS_PCG_GRAPH=0;POMS_PCG_SPEC=1,POMS_PCG_GRAPH=1;POMS_NATIVE_PCG=0" > $O/ab2d.log 2>&1; rc=$?; echo "ab2d rc=$rc"; tail -1 $O/ab2d.log; [ $rc -eq 0 ] || stop ab2d $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_2d -o run -- \
    python3 $R/bench.py --ndim 2 --steps 10 --warmup 3 --no-cpu-baseline) > $O/trace_2d.log 2>&1; rc=$?; echo "trace_2d rc=$rc"; [ $rc -eq 0 ] || stop trace_2d $rc
[ "${2:-}" = "2d" ] && { echo "session done"; exit 0; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_loop -o run -- \
    python3 $R/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 2) > $O/trace_loop.log 2>&1; rc=$?; echo "trace_loop rc=$rc"; [ $rc -eq 0 ] || stop trace_loop $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_planes -o run -- \
    python3 $R/tools/slab_proxy.py --planes 67 --steps 2) > $O/trace_planes.log 2>&1; rc=$?; echo "trace_planes rc=$rc"; [ $rc -eq 0 ] || stop trace_planes $rc
echo "session done"
