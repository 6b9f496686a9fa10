set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_solvers.py -k "native or timing or vcycle" > gpurun_out/pt_spin.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sync_probe.py > gpurun_out/sync_probe2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --ndim 2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench2d_spin.log 2>&1 || exit 1
: > gpurun_out/kb_ord.log
for ord in 0 1 0 1; do
POMS_TILE_ORDER=$ord timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 2 --kinds apply,jacobi --variants 10 | sed "s/^{/{\"ord\": $ord, /" >> gpurun_out/kb_ord.log || exit 1
done
