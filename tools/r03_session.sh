#!/bin/bash
# Round-3 GPU session: GPU suite, smoke, 3D and 2D benches, rocprofv3 kernel stats of
# the 3D bench, the apply's launch series.  Each GPU step has its own time limit and
# a failure stops the session.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03s}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || stop pytest $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || stop smoke $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-200; [ $rc -eq 0 ] || stop bench $rc
timeout -k 10 300 python bench.py --ndim 2 --no-cpu-baseline > $O/bench_2d.log 2>&1; rc=$?; echo "bench2d rc=$rc"; [ $rc -eq 0 ] || stop bench2d $rc
timeout -k 10 200 python tools/kernel_bench.py --cells 512 --p 3 --reps 40 --rounds 2 --variants 10 --kinds apply,jacobi,residual --dump > $O/kb_launch_series.log 2>&1; rc=$?; [ $rc -eq 0 ] || stop kb $rc
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline) > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || stop rocprof $rc
echo "session done"
