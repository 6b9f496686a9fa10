#!/usr/bin/env bash
# Round 6: SQ counters (one --pmc pass) and HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of the
# 2D two-sweep launch and the single v3 sweep (tools/r06/j2_bench.py), each pass its own run.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/j2pmc"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/g$i" -o pmc -- \
      python3 "$ROOT/tools/r06/j2_bench.py" > "$OUT/g$i.log" 2>&1
  rc=$?; echo "group $i rc=$rc"
  [[ $rc -eq 0 ]] || { echo "STOP"; exit $rc; }
done
echo done
