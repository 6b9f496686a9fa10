#!/bin/bash
# Interleaved A/B/... of several builds of the library: tools/kernel_bench.py in
# alternating processes, one per build and round.
#   bash tools/r05/ab_multi.sh <tag> <name=lib.so|name=default,...> <rounds> <kernel_bench args...>
set -u
O=gpurun_out/$1; LIBS=$2; R=$3; shift 3; mkdir -p $O
for r in $(seq 1 $R); do
  for pair in ${LIBS//,/ }; do
    name=${pair%%=*}; lib=${pair#*=}
    if [ "$lib" = default ]; then unset POMS_HIP_LIB; else export POMS_HIP_LIB=$PWD/$lib; fi
    timeout -k 10 200 python tools/kernel_bench.py "$@" > $O/kb_${name}_$r.log 2>&1 || { echo "fail $name $r"; exit 1; }
    echo "$name $r: $(grep -h median_us $O/kb_${name}_$r.log | python -c 'import sys,json; print([(d["kind"], round(d["median_us"],1), round(d["min_us"],1)) for d in map(json.loads, sys.stdin)])')"
  done
done
