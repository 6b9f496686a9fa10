#!/usr/bin/env bash
# SQ counters (one rocprofv3 --pmc pass per group) of kernel_bench launches.
# Usage: tools/pmc_sq.sh <tag> <kernel_bench args...>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
tag="$1"; shift
OUT="$ROOT/gpurun_out/pmc_$tag"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS"
gi=0
for grp in "$G1" "$G2" ${EXTRA_GROUPS:-}; do
  gi=$((gi+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/g$gi" -o pmc -- \
      python3 "$ROOT/tools/kernel_bench.py" --rounds 1 --reps 2 "$@" > "$OUT/g$gi.log" 2>&1
  rc=$?; echo "group $gi rc=$rc"
  [[ $rc -eq 0 ]] || { echo "STOP"; exit $rc; }
done
echo done
