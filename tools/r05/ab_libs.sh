#!/bin/bash
# Interleaved A/B of two builds of the library: tools/kernel_bench.py in alternating
# processes, POMS_HIP_LIB pointing at the old build (abtmp/libpoms_hip_old.so, linked
# by hand from the old kron_v5 object and the current other objects).
#   bash tools/r05/ab_libs.sh <tag> <kernel_bench args...>
set -u
O=gpurun_out/$1; shift; mkdir -p $O
for r in 1 2 3; do
  for lib in old new; do
    if [ $lib = old ]; then export POMS_HIP_LIB=$PWD/abtmp/libpoms_hip_old.so; else unset POMS_HIP_LIB; fi
    timeout -k 10 200 python tools/kernel_bench.py "$@" > $O/kb_${lib}_$r.log 2>&1 || { echo "fail $lib $r"; exit 1; }
    echo "$lib $r: $(grep -h median_us $O/kb_${lib}_$r.log | python -c 'import sys,json; print([(d["kind"], round(d["median_us"],1), round(d["min_us"],1)) for d in map(json.loads, sys.stdin)])')"
  done
done
