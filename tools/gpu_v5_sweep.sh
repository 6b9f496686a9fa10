set -u
mkdir -p gpurun_out
timeout -k 10 500 python tools/kernel_bench.py --cells 512 --p 3 --reps 8 --rounds 3 --variants 10,103,104,105,106 --kinds apply,residual,jacobi > gpurun_out/kb_v5_cp.log 2>&1 || exit 1
echo ok
