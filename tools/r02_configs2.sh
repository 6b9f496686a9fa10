#!/bin/bash
# BASELINE configs 3 and 5 on the closing build: kernels (no flush, as
# profiles/r02/configs/kb_p5_waves8.log) and V-cycles.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/configs2; mkdir -p $O
timeout -k 10 300 python -u tools/kernel_bench.py --cells 256 --p 5 --reps 10 --rounds 3 --variants 10 --kinds apply,jacobi,from_zero > $O/kb_p5.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/kernel_bench.py --cells 256 --p 2 --reps 10 --rounds 3 --variants 10 --kinds apply,jacobi,from_zero > $O/kb_p2.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --p 5 --cells 256 --no-cpu-baseline > $O/bench_p5.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --p 2 --cells 256 --no-cpu-baseline > $O/bench_p2.log 2>&1 || exit 1
for f in $O/kb_p5.log $O/kb_p2.log; do echo "== $f"; grep -h GBps $f | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['variant'], d['kind'], round(d['median_us'],1), round(d['min_us'],1))"; done
for f in $O/bench_p5.log $O/bench_p2.log; do tail -1 $f | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],2), round(d['value']/1e6,1), round(d['roofline']['avg_launch_us'],1), d['roofline']['kernel'])"; done
