set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "10" > gpurun_out/pt_v5.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pt_v5.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 2 --variants 7,9,10 --kinds apply,residual,jacobi > gpurun_out/kb_v5.log 2>&1
rc=$?; echo "kb rc=$rc"; tail -12 gpurun_out/kb_v5.log
