#!/bin/bash
# One-rank proxies of the 8-GPU V-cycle (tools/slab_proxy.py): the halo-free slab grid,
# and ranks 1 (two neighbour sides) and 0 (one) of the real 515^3 split with the
# exchanges and sums looped back through a one-rank RCCL communicator; rocprofv3 stats
# of the rank-1 loopback run.  Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03proxy}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 300 python tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 5 > $O/proxy_loop_r1.log 2>&1; rc=$?; echo "loop r1 rc=$rc"; tail -1 $O/proxy_loop_r1.log | cut -c1-400; [ $rc -eq 0 ] || stop loop1 $rc
timeout -k 10 300 python tools/slab_proxy.py --loopback-rank 0 --world 8 --steps 5 > $O/proxy_loop_r0.log 2>&1; rc=$?; echo "loop r0 rc=$rc"; tail -1 $O/proxy_loop_r0.log | cut -c1-400; [ $rc -eq 0 ] || stop loop0 $rc
timeout -k 10 300 python tools/slab_proxy.py --planes 67 --steps 5 > $O/proxy_67.log 2>&1; rc=$?; echo "p67 rc=$rc"; tail -1 $O/proxy_67.log | cut -c1-400; [ $rc -eq 0 ] || stop p67 $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3) > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || stop rocprof $rc
echo "proxy session done"
