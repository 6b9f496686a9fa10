#!/bin/bash
# 2D p = 3 1024^2 V-cycle with the Jacobi sweeps on v3 (default) or v4, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03jac2d; mkdir -p $O
for rnd in 1 2 3; do for v in 9 7; do
  POMS_JAC2D_VARIANT=$v timeout -k 10 200 python bench.py --ndim 2 --no-cpu-baseline --steps 40 > $O/b_v${v}_r$rnd.log 2>&1 || { echo STOP; exit 1; }
  echo "v$v r$rnd $(python3 -c "import json; d=[json.loads(l) for l in open('$O/b_v${v}_r$rnd.log') if l.startswith('{')][-1]; print(round(d['ms_per_step'],3))")"
done; done
