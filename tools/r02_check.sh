set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "from_zero" > gpurun_out/pt_j0.log 2>&1 || exit 1
: > gpurun_out/kb_j0.log
timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 2 --kinds from_zero,jacobi --variants 9,10 >> gpurun_out/kb_j0.log 2>&1 || exit 1
for P in 2 1; do
timeout -k 10 300 python tools/kernel_bench.py --cells 256 --p $P --reps 10 --rounds 2 --kinds from_zero --variants 9,10 --flush >> gpurun_out/kb_j0.log 2>&1 || exit 1
done
