#!/bin/bash
# SQ counters and HBM traffic of the 3D p = 5 apply and Jacobi sweep at 256^3 (the
# BASELINE p = 5 config), and of the rewritten p = 3 two-sweeps-from-zero launch at
# 515^3: one rocprofv3 --pmc pass per counter group, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03pmc}; mkdir -p $O
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
for k in apply jacobi; do
  bash tools/pmc_sq.sh p5_$k --cells 256 --p 5 --kinds $k > $O/sq_p5_$k.log 2>&1; rc=$?; echo "sq p5 $k rc=$rc"; [ $rc -eq 0 ] || stop sq$k $rc
  POMS_PMC_DOF=17779581 bash tools/pmc_traffic.sh p5_$k "kron_v5_kernel<5" --cells 256 --p 5 --kinds $k > $O/traffic_p5_$k.log 2>&1; rc=$?; echo "traffic p5 $k rc=$rc"; [ $rc -eq 0 ] || stop tr$k $rc
  timeout -k 10 200 python tools/kernel_bench.py --cells 256 --p 5 --reps 20 --rounds 2 --kinds $k > $O/kb_p5_$k.log 2>&1; rc=$?; [ $rc -eq 0 ] || stop kb$k $rc
done
bash tools/pmc_sq.sh j0 --cells 512 --p 3 --kinds from_zero > $O/sq_j0.log 2>&1; rc=$?; echo "sq j0 rc=$rc"; [ $rc -eq 0 ] || stop sqj0 $rc
bash tools/pmc_traffic.sh j0 "kron_v5_kernel<3, 3" --cells 512 --p 3 --kinds from_zero > $O/traffic_j0.log 2>&1; rc=$?; echo "traffic j0 rc=$rc"; [ $rc -eq 0 ] || stop trj0 $rc
echo "pmc done"
