set -u
mkdir -p gpurun_out
timeout -k 10 500 python tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 3 --variants 10,109 --kinds apply,residual,jacobi > gpurun_out/kb_v5_nt8.log 2>&1 || exit 1
echo ok
