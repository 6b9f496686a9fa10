#!/bin/bash
# pcg vector updates at 515^3 for several grid caps (POMS_VEC_BLOCKS), two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
for rnd in 1 2; do for nb in 4096 65536; do
  POMS_VEC_BLOCKS=$nb timeout -k 10 120 python tools/vec_bench.py --reps 30 2>&1 | grep -v amdgpu.ids >> gpurun_out/vec_blocks.log || exit 1
done; done
cat gpurun_out/vec_blocks.log
