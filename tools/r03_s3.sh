#!/bin/bash
# Round-3 session 3: parity of the rewritten two-sweeps-from-zero kernel and of the
# split operator call with its boundary launch on the communication stream; A/B of
# the from-zero launch against the previous library (poms_amd/exp/lib_base.so) on
# one box; the loopback proxy with the boundary launch on / off the communication
# stream; the 3D bench.  Each GPU step has its own time limit; a failure stops.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03s3}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_dist.py tests/test_gpu_solvers.py \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || stop pytest $rc
for rnd in 1 2; do
  for L in poms_amd/exp/lib_base.so poms_amd/libpoms_hip.so; do
    POMS_HIP_LIB=$PWD/$L timeout -k 10 200 python tools/kernel_bench.py --cells 512 --p 3 --reps 30 --rounds 1 --kinds from_zero,jacobi,apply \
      2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $L .so) r$rnd |" >> $O/kb_ab.log
    rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || stop kb $rc
  done
done
cut -c1-160 $O/kb_ab.log
for cs in 1 0; do
  POMS_BOUNDARY_ON_CS=$cs timeout -k 10 300 python tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 5 > $O/proxy_loop_r1_cs$cs.log 2>&1
  rc=$?; echo "proxy cs=$cs rc=$rc"; tail -1 $O/proxy_loop_r1_cs$cs.log | cut -c1-250; [ $rc -eq 0 ] || stop proxy$cs $rc
done
timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-300; [ $rc -eq 0 ] || stop bench $rc
echo "session done"
