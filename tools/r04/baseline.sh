#!/bin/bash
# Round-4 first session: the committed tree's kernel medians and the 3D bench on this box.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r04base}; mkdir -p $O
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 40 --rounds 2 --kinds apply,jacobi,from_zero > $O/kb.log 2>&1; rc=$?; echo "kb rc=$rc"; tail -8 $O/kb.log; [ $rc -eq 0 ] || stop kb $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-400; [ $rc -eq 0 ] || stop bench $rc
echo "session done"
