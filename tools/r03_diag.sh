#!/bin/bash
# J0 with and without its running sums (variant 110, timing only) beside the apply+dot
# launch, and the 2D p = 3 1024^2 sweep / apply over the kernel variants.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 20 --rounds 2 --kinds from_zero --variants 10,110 > gpurun_out/kb_j0diag.log 2>&1 && \
timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 20 --rounds 2 --kinds apply_dot,apply >> gpurun_out/kb_j0diag.log 2>&1 && \
timeout -k 10 200 python tools/kernel_bench.py --ndim 2 --cells 1024 --p 3 --reps 100 --rounds 2 --kinds jacobi,apply --variants 9,7,4,0 > gpurun_out/kb_2d_variants.log 2>&1
rc=$?
cut -c1-170 gpurun_out/kb_j0diag.log gpurun_out/kb_2d_variants.log | grep -v amdgpu.ids
exit $rc
