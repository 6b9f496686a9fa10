#!/bin/bash
# Tile order 0 (t2 fastest) vs 1 (t1 fastest: vertical neighbours on one XCD) for the
# 515^3 apply and Jacobi sweep: HBM traffic (separate FETCH / WRITE passes) and
# timings, one box.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03order; mkdir -p $O
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
for ord in 0 1; do
  for k in apply jacobi; do
    POMS_TILE_ORDER=$ord bash tools/pmc_traffic.sh ord${ord}_$k "kron_v5_kernel<3" --cells 512 --p 3 --kinds $k > $O/traffic_ord${ord}_$k.log 2>&1; rc=$?; [ $rc -eq 0 ] || stop tr $rc
    echo "ord $ord $k $(python3 -c "import json; d=json.load(open('gpurun_out/pmct_ord${ord}_$k/traffic.json')); print(round(d['bytes_per_dof'],2))")"
  done
done
for rnd in 1 2; do for ord in 0 1; do
  POMS_TILE_ORDER=$ord timeout -k 10 200 python tools/kernel_bench.py --cells 512 --p 3 --reps 20 --rounds 1 --kinds apply,jacobi 2>&1 | grep -v amdgpu.ids | sed "s/^/ord$ord r$rnd /" | cut -c1-130 | tee -a $O/kb.log
done; done
