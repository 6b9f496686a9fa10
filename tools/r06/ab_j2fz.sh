#!/usr/bin/env bash
# Round 6: the 2D bench with the three-sweeps-from-zero launch on / off (POMS_J2FZ), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=gpurun_out/ab_j2fz; mkdir -p $O
for i in 1 2 3; do
  for v in 1 0; do
    POMS_J2FZ=$v timeout -k 10 200 python bench.py --ndim 2 --no-cpu-baseline > $O/b_${v}_$i.log 2>&1 || { echo "rc=$?"; exit 1; }
    echo "J2FZ=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_$i.log)"
  done
done
