#!/bin/bash
# Round-5 session 11: 2D epilogue operands issued with the x rows (v3, IS3D=false):
# A/B of the libraries on kernel_bench and the 2D V-cycle, plus 2D GPU tests.
set -o pipefail
O=gpurun_out/s11
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "2d or two_d or 2D" --timeout 120 --timeout-method thread > $O/t_2d.log 2>&1 || exit 1
for r in 1 2; do
  for lib in pre2d 2dearly; do
    POMS_HIP_LIB=poms_amd/exp/lib_$lib.so timeout -k 10 200 python tools/kernel_bench.py --ndim 2 --cells 1024 --reps 50 --rounds 2 --kinds jacobi,apply_dot,residual > $O/kb_${lib}_$r.log 2>&1 || exit 2
  done
done
for r in 1 2; do
  for lib in pre2d 2dearly; do
    POMS_HIP_LIB=poms_amd/exp/lib_$lib.so timeout -k 10 300 python bench.py --ndim 2 --no-cpu-baseline > $O/bench2d_${lib}_$r.log 2>&1 || exit 3
  done
done
echo done
