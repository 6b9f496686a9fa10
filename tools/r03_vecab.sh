#!/bin/bash
# In-cycle A/B of the flat vector kernels' grid (POMS_VEC_BLOCKS=4096 vs the 65536
# default) on one box: parity of the vector / solver tests, 3D bench interleaved
# twice, rocprofv3 kernel statistics of the default.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03vecab}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solvers.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || stop pytest $rc
for rnd in 1 2; do for nb in 4096 65536; do
  POMS_VEC_BLOCKS=$nb timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $O/bench_nb${nb}_r$rnd.log 2>&1; rc=$?; [ $rc -eq 0 ] || stop bench $rc
  echo "nb=$nb r$rnd $(python3 -c "import json,sys; d=[json.loads(l) for l in open('$O/bench_nb${nb}_r$rnd.log') if l.startswith('{')][-1]; print(round(d['ms_per_step'],2), round(d['roofline']['avg_launch_us'],1))")"
done; done
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline) > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
