#!/usr/bin/env bash
# One GPU session on the gpurun box: GPU tests -> smoke -> bench -> rocprofv3 stats.
# Every GPU step has its own time limit; a crash/timeout (exit >= 2 for pytest,
# != 0 otherwise) stops the session so nothing else touches the GPU.
# Usage: tools/gpu_session.sh [tests|bench|prof|all] [extra bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
what="${1:-all}"; shift || true

stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }

if [[ "$what" == "tests" || "$what" == "all" ]]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
  [[ $rc -le 1 ]] || stop "pytest crashed or timed out" $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"
  [[ $rc -eq 0 ]] || stop "smoke failed" $rc
fi
if [[ "$what" == "bench" || "$what" == "all" ]]; then
  timeout -k 10 900 python bench.py "$@" > "$OUT/bench.log" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.log"
  [[ $rc -eq 0 ]] || stop "bench failed" $rc
fi
if [[ "$what" == "prof" || "$what" == "all" ]]; then
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --kron-reps 5 "$@") > "$OUT/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof.log"
  [[ $rc -eq 0 ]] || stop "rocprof failed" $rc
fi
echo "session done"
