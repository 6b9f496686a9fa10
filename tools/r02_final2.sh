#!/usr/bin/env bash
# Round-2 closing session on the committed tree: GPU tests, smoke, bench (3D headline
# with CPU baseline, 2D config), rocprofv3 kernel stats of the bench command, PMC
# traffic of the Jacobi sweep and the apply.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-final2}
mkdir -p $OUT
bash tools/gpu_session.sh tests > $OUT/session_tests.log 2>&1 || { echo "tests stop"; tail -5 $OUT/session_tests.log; exit 1; }
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log $OUT/
tail -3 $OUT/pytest_gpu.log
timeout -k 10 900 python -u bench.py > $OUT/bench.log 2>&1 || exit 1
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --ndim 2 > $OUT/bench_2d.log 2>&1 || exit 1
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline) > $OUT/prof.log 2>&1 || exit 1
bash tools/pmc_traffic.sh j10 "kron_v5_kernel<3, 2, 4, 0, 70," --cells 512 --p 3 --kinds jacobi --variants 10 > $OUT/pmc.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/pmct_j10 "kron_v5_kernel<3, 2, 4, 0, 70," 136590875 $OUT/pmc_traffic_jacobi.json 3 10 > /dev/null
bash tools/pmc_traffic.sh a10 "kron_v5_kernel<3, 0, 4, 0, 6," --cells 512 --p 3 --kinds apply --variants 10 > $OUT/pmc_apply.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/pmct_a10 "kron_v5_kernel<3, 0, 4, 0, 6," 136590875 $OUT/pmc_traffic_apply.json 3 10 > /dev/null
echo done
