#!/usr/bin/env bash
# PMC counter passes (one rocprofv3 run per counter group, --pmc never combined
# with sys/runtime tracing) over the kernel micro-benchmark, then kernel-trace stats.
# Usage: tools/pmc_session.sh <tag> [kernel_bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
tag="${1:-run}"; shift || true
export TMPDIR=/tmp
cd /tmp
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
)
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $g --output-format csv -d "$OUT/${tag}_g$i" -o pmc -- \
      python3 "$ROOT/tools/kernel_bench.py" --rounds 1 --reps 3 "$@" > "$OUT/${tag}_g$i.log" 2>&1
  rc=$?; echo "pmc group $i rc=$rc"
  [[ $rc -eq 0 ]] || { echo "STOP"; exit $rc; }
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${tag}_trace" -o trace -- \
    python3 "$ROOT/tools/kernel_bench.py" --rounds 1 --reps 5 "$@" > "$OUT/${tag}_trace.log" 2>&1
echo "trace rc=$?"
