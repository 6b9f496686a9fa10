#!/bin/bash
# Kernel timings of several libraries on ONE box (interleaved rounds).
# Usage: tools/ab_kb.sh "<kernel_bench args>" lib1.so [lib2.so ...]   ("main" = poms_amd/libpoms_hip.so)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
args="$1"; shift
O=gpurun_out/ab_kb; mkdir -p $O
for rnd in 1 2; do
  for L in "$@"; do
    tag=$(basename $L .so)
    if [ "$L" = main ]; then lib=$PWD/poms_amd/libpoms_hip.so; else lib=$PWD/$L; fi
    POMS_HIP_LIB=$lib timeout -k 10 200 python tools/kernel_bench.py $args 2>&1 | grep -v amdgpu.ids | sed "s/^/$tag r$rnd /" | tee -a $O/kb.log
    rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "STOP rc=$rc"; exit $rc; }
  done
done
