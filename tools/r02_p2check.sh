#!/bin/bash
# Full GPU suite + smoke on the committed tree, then the p = 2 sweeps-from-zero and V-cycle.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p2check; mkdir -p $O
bash tools/gpu_session.sh tests > $O/session_tests.log 2>&1 || { echo "tests stop"; tail -5 $O/session_tests.log; exit 1; }
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log $O/
tail -1 $O/pytest_gpu.log; tail -1 $O/smoke.log
timeout -k 10 300 python -u tools/kernel_bench.py --cells 256 --p 2 --reps 10 --rounds 3 --variants 9,10 --kinds from_zero > $O/kb_p2.log 2>&1 || exit 1
grep -h GBps $O/kb_p2.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['variant'], d['kind'], round(d['median_us'],1), round(d['min_us'],1))"
timeout -k 10 400 python -u bench.py --p 2 --cells 256 --no-cpu-baseline > $O/bench_p2.log 2>&1 || exit 1
tail -1 $O/bench_p2.log | cut -c1-200
