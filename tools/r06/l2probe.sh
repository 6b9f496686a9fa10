#!/bin/bash
# Round 6: where the apply's x over-read comes from. HBM traffic (separate FETCH / WRITE
# passes) and interleaved times of the production apply (variant 10, dispatch table on
# and off) and its memory-only build (variant 101, the same tiles / DMA ring, no arithmetic).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/l2probe
mkdir -p $O
timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 3 --variants 10,101 --kinds apply > $O/kb.log 2>&1
rc=$?; echo "kb rc=$rc"; cat $O/kb.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
POMS_V5_SCHED=0 timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 3 --variants 10,101 --kinds apply > $O/kb_s0.log 2>&1
rc=$?; echo "kb s0 rc=$rc"; cat $O/kb_s0.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
for v in 10 101; do
  for s in 1 0; do
    POMS_V5_SCHED=$s bash tools/pmc_traffic.sh v${v}_s$s kron_v5 --cells 512 --p 3 --variants $v --kinds apply > $O/pmc_v${v}_s$s.log 2>&1
    rc=$?; echo "v$v s$s pmc rc=$rc"; grep bytes_per_dof gpurun_out/pmct_v${v}_s$s/traffic.json; [ $rc -eq 0 ] || exit $rc
  done
done
