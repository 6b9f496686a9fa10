#!/usr/bin/env bash
# Round 6: the two-sweep launch's tile shapes (POMS_J2_TILE=R,RE), parity and timing
# per shape, two passes interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=gpurun_out/j2tiles; mkdir -p $O
for pass in 1 2; do
  for t in 6,4 7,5 6,5 5,4 5,3; do
    POMS_J2_TILE=$t timeout -k 10 120 python tools/r06/j2_diag2.py > $O/parity_${t/,/_}_$pass.log 2>&1 || { echo "parity $t rc=$?"; exit 1; }
    bad=$(grep -c "bad 0 " $O/parity_${t/,/_}_$pass.log)
    POMS_J2_TILE=$t timeout -k 10 120 python tools/r06/j2_bench.py > $O/bench_${t/,/_}_$pass.log 2>&1 || { echo "bench $t rc=$?"; exit 1; }
    echo "pass $pass tile $t parity-clean-runs $bad: $(grep -h spline $O/bench_${t/,/_}_$pass.log)"
  done
done
