#!/bin/bash
# v7 apply: parity tests, then v5 vs v7 interleaved on one box (515^3, p = 3).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r04v7}; mkdir -p $O
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_v7.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_v7.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest_v7.log; [ $rc -eq 0 ] || stop pytest $rc
timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 40 --rounds 3 --variants 10,11 --kinds apply,jacobi,residual,apply_dot > $O/kb_v5_v7.log 2>&1; rc=$?; echo "kb rc=$rc"; cat $O/kb_v5_v7.log | cut -c1-200; [ $rc -eq 0 ] || stop kb $rc
echo "session done"
