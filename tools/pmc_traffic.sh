#!/usr/bin/env bash
# HBM traffic (separate --pmc FETCH_SIZE / WRITE_SIZE passes) of one kernel_bench kind/variant.
# Usage: tools/pmc_traffic.sh <tag> <kernel-substring> <kernel_bench args...>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
tag="$1"; sub="$2"; shift 2
OUT="$ROOT/gpurun_out/pmct_$tag"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
gi=0
for grp in FETCH_SIZE WRITE_SIZE; do
  gi=$((gi+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/g$gi" -o pmc -- \
      python3 "$ROOT/tools/kernel_bench.py" --rounds 1 --reps 3 "$@" > "$OUT/g$gi.log" 2>&1
  rc=$?; echo "$tag group $gi rc=$rc"
  [[ $rc -eq 0 ]] || { echo "STOP"; exit $rc; }
done
python3 "$ROOT/tools/pmc_traffic.py" "$OUT" "$sub" ${POMS_PMC_DOF:-136590875} "$OUT/traffic.json" > /dev/null && cat "$OUT/traffic.json"
