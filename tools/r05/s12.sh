#!/bin/bash
# Round-5 session 12: axis-0 chunk sweep of the 515^3 p=3 launches on the round-5
# kernels (the two-sweeps-from-zero launch halves the model's 172-plane chunk; the
# choice dates from round 3).
set -o pipefail
O=gpurun_out/s12
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  timeout -k 10 400 python tools/kernel_bench.py --cells 512 --reps 10 --rounds 2 --kinds from_zero --chunks 0,57,65,75,86,103,129,172 > $O/kb_j0_chunks_$r.log 2>&1 || exit 1
  timeout -k 10 400 python tools/kernel_bench.py --cells 512 --reps 10 --rounds 2 --kinds jacobi,apply --chunks 0,86,103,129,172 > $O/kb_jac_chunks_$r.log 2>&1 || exit 2
done
echo done
