#!/bin/bash
# v7 apply diagnosis: memory-only / arithmetic-only builds beside v5 and v7 (one box,
# interleaved), SQ counters and HBM traffic of the v7 apply.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r04v7diag}; mkdir -p $O
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 400 python tools/kernel_bench.py --cells 512 --p 3 --reps 30 --rounds 3 --variants 10,11,101,121,122,123,124 --kinds apply > $O/kb_modes.log 2>&1; rc=$?; echo "kb rc=$rc"; cut -c1-160 $O/kb_modes.log; [ $rc -eq 0 ] || stop kb $rc
timeout -k 10 400 python tools/kernel_bench.py --cells 512 --p 3 --reps 30 --rounds 2 --variants 11 --chunks 0,172,129,103,86,58 --kinds apply > $O/kb_chunks.log 2>&1; rc=$?; echo "kbc rc=$rc"; cut -c1-160 $O/kb_chunks.log; [ $rc -eq 0 ] || stop kbc $rc
timeout -k 10 300 bash tools/pmc_sq.sh v7apply --cells 512 --p 3 --variants 11 --kinds apply > $O/sq.log 2>&1; rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || stop sq $rc
timeout -k 10 300 bash tools/pmc_traffic.sh v7apply kron_v7 --cells 512 --p 3 --variants 11 --kinds apply > $O/traffic.log 2>&1; rc=$?; echo "traffic rc=$rc"; tail -3 $O/traffic.log; [ $rc -eq 0 ] || stop traffic $rc
echo "session done"
