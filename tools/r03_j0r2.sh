#!/bin/bash
# Two sweeps from zero, 8 waves x 2 rows (this tree) against 16 waves x 1 row
# (poms_amd/exp/lib_j0r1.so): outputs compared at 100^3 and 515^3, timings A/B.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03j0r2; mkdir -p $O
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
for c in 100 512; do
  POMS_HIP_LIB=$PWD/poms_amd/exp/lib_j0r1.so timeout -k 10 200 python tools/j0_dump.py $O/r1_$c.npz $c || stop r1 $?
  timeout -k 10 200 python tools/j0_dump.py $O/r2_$c.npz $c || stop r2 $?
  python3 -c "
import numpy as np
a=np.load('$O/r1_$c.npz'); b=np.load('$O/r2_$c.npz')
print('cells $c rel', np.linalg.norm(a['y']-b['y'])/np.linalg.norm(a['y']), 'norms', abs(a['m1']-b['m1'])/a['m1'], abs(a['m2']-b['m2'])/a['m2'], int(a['variant']), int(b['variant']))"
done
for rnd in 1 2; do for L in poms_amd/exp/lib_j0r1.so poms_amd/libpoms_hip.so; do
  POMS_HIP_LIB=$PWD/$L timeout -k 10 200 python tools/kernel_bench.py --cells 512 --p 3 --reps 20 --rounds 1 --kinds from_zero 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $L .so) r$rnd |" | cut -c1-150 | tee -a $O/kb.log
done; done
