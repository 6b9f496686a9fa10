#!/bin/bash
# Two sweeps from zero with its running sums added by LDS atomics (this tree) against
# the read-modify-write build (poms_amd/exp/lib_j0rmw.so): J0 parity tests, A/B timing.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03j0add; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_solvers.py -m gpu -x -q -k "zero or fullsize or native or vcycle" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rnd in 1 2 3; do for L in poms_amd/exp/lib_j0rmw.so poms_amd/libpoms_hip.so; do
  POMS_HIP_LIB=$PWD/$L timeout -k 10 200 python tools/kernel_bench.py --cells 512 --p 3 --reps 20 --rounds 1 --kinds from_zero 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $L .so) r$rnd |" | cut -c1-150 >> $O/kb.log || exit 1
done; done
cat $O/kb.log
