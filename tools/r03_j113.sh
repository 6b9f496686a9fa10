#!/bin/bash
# Jacobi sweep at 515^3: production build (variant 10) vs streaming the x rows no
# other tile reads (variant 113): HBM traffic (FETCH / WRITE passes) and timings, one box.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03j113; mkdir -p $O
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
for v in 10 113; do
  bash tools/pmc_traffic.sh j$v "kron_v5_kernel<3, 2" --cells 512 --p 3 --kinds jacobi --variants $v > $O/traffic_$v.log 2>&1; rc=$?; [ $rc -eq 0 ] || stop tr $rc
  echo "variant $v $(python3 -c "import json; d=json.load(open('gpurun_out/pmct_j$v/traffic.json')); print(round(d['bytes_per_dof'],2), round(d['hbm_read_bytes_per_launch']/1e9,3))")"
done
timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 20 --rounds 3 --kinds jacobi --variants 10,113 2>&1 | grep -v amdgpu.ids | cut -c1-140 | tee $O/kb.log
