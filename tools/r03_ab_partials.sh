#!/bin/bash
# A/B on one box: host-added partials (POMS_HOST_PARTIALS = max blocks) vs the device
# reduction launch (0), 2D and 3D V-cycles, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03ab}; mkdir -p $O
for rep in 1 2; do
  for m in 0 2048; do
    POMS_HOST_PARTIALS=$m timeout -k 10 200 python bench.py --ndim 2 --no-cpu-baseline --steps 40 > $O/b2d_m${m}_r$rep.log 2>&1 || exit 1
    echo "2D m=$m rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $O/b2d_m${m}_r$rep.log)"
  done
done
for rep in 1 2; do
  for m in 0 512; do
    POMS_HOST_PARTIALS=$m timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > $O/b3d_m${m}_r$rep.log 2>&1 || exit 1
    echo "3D m=$m rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $O/b3d_m${m}_r$rep.log)"
  done
done
