#!/bin/bash
# GPU parity of the distributed / native-pcg paths, then the rank-1 loopback proxy
# with RCCL's kernels capped at 4 / 8 / 16 / 32 workgroups (POMS_COMM_CTAS) and uncapped.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03proxy2}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 600 python -u -m pytest tests/test_dist.py tests/test_gpu_solvers.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || stop pytest $rc
for c in 0 32 16 8 4; do
  POMS_COMM_CTAS=$c timeout -k 10 300 python tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 5 > $O/proxy_loop_r1_ctas$c.log 2>&1; rc=$?; echo "ctas $c rc=$rc"; tail -1 $O/proxy_loop_r1_ctas$c.log | cut -c1-250; [ $rc -eq 0 ] || stop loop$c $rc
done
(cd /tmp && POMS_COMM_CTAS=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3) > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || stop rocprof $rc
echo "done"
