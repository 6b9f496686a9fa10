#!/bin/bash
# memory-only build of the v5 apply (variant 101) with the production y-store policy: traffic
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/m1probe; mkdir -p $O
export POMS_HIP_LIB=$PWD/ab/lib_m1nt.so
timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 2 --variants 10,101 --kinds apply > $O/kb.log 2>&1
rc=$?; echo "kb rc=$rc"; cut -c1-160 $O/kb.log; [ $rc -eq 0 ] || exit $rc
for v in 101; do
  bash tools/pmc_traffic.sh m1nt_v$v kron_v5 --cells 512 --p 3 --variants $v --kinds apply > $O/pmc_v$v.log 2>&1
  rc=$?; echo "v$v pmc rc=$rc"; grep -E "bytes_per_dof|read_bytes" gpurun_out/pmct_m1nt_v$v/traffic.json; [ $rc -eq 0 ] || exit $rc
done
