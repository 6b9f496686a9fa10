#!/bin/bash
# GPU parity of the comm / distributed / native-pcg paths, then the loopback proxies
# (rank 1 with RCCL's kernels uncapped and capped at 8 workgroups, rank 0) and a
# rocprofv3 kernel trace of the rank-1 run.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03proxy3}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_dist.py tests/test_gpu_solvers.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || stop pytest $rc
for c in 0 8; do
  POMS_COMM_CTAS=$c timeout -k 10 300 python tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 5 > $O/proxy_loop_r1_ctas$c.log 2>&1; rc=$?; echo "ctas $c rc=$rc"; tail -1 $O/proxy_loop_r1_ctas$c.log | cut -c1-250; [ $rc -eq 0 ] || stop loop$c $rc
done
timeout -k 10 300 python tools/slab_proxy.py --loopback-rank 0 --world 8 --steps 5 > $O/proxy_loop_r0.log 2>&1; rc=$?; echo "r0 rc=$rc"; tail -1 $O/proxy_loop_r0.log | cut -c1-250; [ $rc -eq 0 ] || stop loop0 $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3) > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || stop rocprof $rc
echo "done"
