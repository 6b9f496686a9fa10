#!/bin/bash
# Round-5 experiment record: the three POMS_V5_PRIO runtime modes of a one-off build
# (0 none, 1 priority dropped after the axis-1 pass, 2 dropped before the axis-0
# scatter), interleaved in alternating processes.  Mode 2 is now compiled in
# unconditionally and the variable is gone (profiles/r05/prio/runtime_modes.log).
set -u
O=gpurun_out/s33; mkdir -p $O
for r in 1 2; do
  for m in 0 1 2; do
    POMS_V5_PRIO=$m timeout -k 10 200 python tools/kernel_bench.py --kinds apply,jacobi,from_zero --rounds 2 --reps 15 > $O/kb_p${m}_$r.log 2>&1 || exit 1
    echo "prio $m $r: $(grep -h median_us $O/kb_p${m}_$r.log | python -c 'import sys,json; print([(d["kind"], round(d["median_us"],1), round(d["min_us"],1)) for d in map(json.loads, sys.stdin)])')"
  done
done
