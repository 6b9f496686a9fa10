#!/bin/bash
# v7 vs v5 on one box after the LDS-conflict fixes: parity, kernel medians, SQ counters.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r04v7c}; mkdir -p $O
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_v7.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_v7.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_v7.log; [ $rc -eq 0 ] || stop pytest $rc
timeout -k 10 400 python tools/kernel_bench.py --cells 512 --p 3 --reps 30 --rounds 3 --variants 10,11 --chunks 0,103 --kinds apply,jacobi > $O/kb.log 2>&1; rc=$?; echo "kb rc=$rc"; cut -c1-150 $O/kb.log; [ $rc -eq 0 ] || stop kb $rc
timeout -k 10 300 bash tools/pmc_sq.sh v7c --cells 512 --p 3 --variants 11 --kinds apply > $O/sq.log 2>&1; rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || stop sq $rc
echo "session done"
