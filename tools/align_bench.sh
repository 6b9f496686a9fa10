#!/usr/bin/env bash
# Row-pitch alignment x tile output width, 515^3 p=3 (variants 7 = v4, 9 = v3 whole-array).
set -u
OUT=gpurun_out/align; mkdir -p $OUT
timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 8 --rounds 3 --variants 7,9 --tile-cols 0,48 --kinds apply,residual,jacobi > $OUT/aligned.log 2>&1 || exit 1
timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 8 --rounds 3 --variants 7,9 --tile-cols 0,48 --kinds apply,residual,jacobi --no-align > $OUT/unaligned.log 2>&1 || exit 1
echo ok
