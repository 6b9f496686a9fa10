#!/bin/bash
# v5 two-sweeps-from-zero (p <= 2): parity under variants 8/9/10, then timing v9 vs v10
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "from_zero or fused_dot or fused_inner" > gpurun_out/pt_j0.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pt_j0.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/kernel_bench.py --cells 256 --p 2 --reps 10 --rounds 3 --variants 9,10 --kinds from_zero,jacobi,apply > gpurun_out/kb_j0_p2.log 2>&1
rc=$?; echo "kb p2 rc=$rc"; tail -8 gpurun_out/kb_j0_p2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/kernel_bench.py --cells 256 --p 1 --reps 10 --rounds 3 --variants 9,10 --kinds from_zero,jacobi > gpurun_out/kb_j0_p1.log 2>&1
rc=$?; echo "kb p1 rc=$rc"; tail -6 gpurun_out/kb_j0_p1.log
exit $rc
