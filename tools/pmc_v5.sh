#!/usr/bin/env bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE; separate --pmc passes) and SQ counters of the
# default operator kernels at 515^3 p=3 (aligned layout), one rocprofv3 run per group.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc5"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS"
for kind in ${KINDS:-apply jacobi}; do
  gi=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "$G1" "$G2"; do
    gi=$((gi+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/${kind}_g$gi" -o pmc -- \
        python3 "$ROOT/tools/kernel_bench.py" --rounds 1 --reps 2 --variants ${VARIANT:-8} --kinds $kind --cells 512 --p 3 \
        > "$OUT/${kind}_g$gi.log" 2>&1
    rc=$?; echo "$kind group $gi rc=$rc"
    [[ $rc -eq 0 ]] || { echo "STOP"; exit $rc; }
  done
done
echo done
