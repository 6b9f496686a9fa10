#!/usr/bin/env bash
# SQ counter passes over kernel_bench for a list of kernel variants (one rocprofv3 run per
# counter group and variant; --pmc only with --output-format, never with tracing).
# Usage: tools/pmc_variants.sh "<variants>" <kinds> [kernel_bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
variants="$1"; kinds="$2"; shift 2
export TMPDIR=/tmp
cd /tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS"
for v in $variants; do
  gi=0
  for grp in "$G1" "$G2" "FETCH_SIZE" "WRITE_SIZE"; do
    gi=$((gi+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/v${v}_g$gi" -o pmc -- \
        python3 "$ROOT/tools/kernel_bench.py" --rounds 1 --reps 2 --variants "$v" --kinds "$kinds" "$@" \
        > "$OUT/v${v}_g$gi.log" 2>&1
    rc=$?; echo "variant $v group $gi rc=$rc"
    [[ $rc -eq 0 ]] || { echo "STOP"; exit $rc; }
  done
done
echo done
