#!/bin/bash
# V-cycles of the other BASELINE configs (3D p = 2 and p = 5 at 256^3) on the
# committed tree.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03configs; mkdir -p $O
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
for p in 2 5; do
  timeout -k 10 300 python bench.py --p $p --cells 256 --steps 5 --no-cpu-baseline > $O/bench_p${p}_256.log 2>&1; rc=$?; [ $rc -eq 0 ] || stop p$p $rc
  echo "p=$p $(python3 -c "import json; d=[json.loads(l) for l in open('$O/bench_p${p}_256.log') if l.startswith('{')][-1]; print(round(d['ms_per_step'],2), round(d['value']/1e6,1), round(d['roofline']['avg_launch_us'],1), round(d['kron_spmv']['median_launch_us'],1))")"
done
