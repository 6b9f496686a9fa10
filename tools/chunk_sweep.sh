#!/usr/bin/env bash
# Axis-0 chunk-length sweep (workgroup count vs halo re-reads) for the v3/v4 kernels.
set -u
OUT=gpurun_out/chunks; mkdir -p $OUT
timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 8 --rounds 3 --variants 7,9 --chunks 0,86 --kinds apply,residual,jacobi > $OUT/512p3_auto.log 2>&1 || exit 1
timeout -k 10 300 python tools/kernel_bench.py --cells 256 --p 5 --reps 8 --rounds 3 --variants 7,9 --chunks 0 --kinds apply,residual,jacobi --flush > $OUT/256p5_auto.log 2>&1 || exit 1
timeout -k 10 300 python tools/kernel_bench.py --cells 256 --p 2 --reps 8 --rounds 3 --variants 7,9 --chunks 0 --kinds apply,residual,jacobi --flush > $OUT/256p2_auto.log 2>&1 || exit 1
echo ok
