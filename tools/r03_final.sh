#!/bin/bash
# Round-3 closing session on the committed tree: the GPU suite, smoke, the 3D and 2D
# benches, rocprofv3 kernel statistics of both benches, and the loopback proxy of
# rank 1 of 8.  Each GPU step has its own time limit; a failure stops the session.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03final}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || stop pytest $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || stop smoke $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-200; [ $rc -eq 0 ] || stop bench $rc
timeout -k 10 300 python bench.py --ndim 2 --no-cpu-baseline > $O/bench_2d.log 2>&1; rc=$?; echo "bench2d rc=$rc"; [ $rc -eq 0 ] || stop bench2d $rc
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline) > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || stop rocprof $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof2d -o run -- python3 $GRAFT_REPO_ROOT/bench.py --ndim 2 --steps 10 --warmup 3 --no-cpu-baseline) > $O/prof2d.log 2>&1
rc=$?; echo "rocprof2d rc=$rc"; [ $rc -eq 0 ] || stop rocprof2d $rc
timeout -k 10 300 python tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 5 > $O/proxy_loop_r1.log 2>&1; rc=$?; echo "proxy rc=$rc"; tail -1 $O/proxy_loop_r1.log | cut -c1-200; [ $rc -eq 0 ] || stop proxy $rc
echo "session done"
