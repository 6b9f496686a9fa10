#!/usr/bin/env bash
# Kernel timings (default operator variant) for every BASELINE.json GPU config.
# Small configs (working set <= MALL) are measured with a cache flush before each launch.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/configs"
mkdir -p "$OUT"
run() { timeout -k 10 300 python "$ROOT/tools/kernel_bench.py" "$@"; }
run --ndim 2 --cells 1024 --p 3 --reps 10 --rounds 2 --kinds apply,residual,jacobi,dot --flush --json "$OUT/2d_p3_1024.json" > "$OUT/2d_p3_1024.log" 2>&1 || exit 1
run --ndim 3 --cells 256 --p 2 --reps 10 --rounds 2 --kinds apply,residual,jacobi,dot --flush --json "$OUT/3d_p2_256.json" > "$OUT/3d_p2_256.log" 2>&1 || exit 1
run --ndim 3 --cells 256 --p 5 --reps 10 --rounds 2 --kinds apply,residual,jacobi,dot --flush --json "$OUT/3d_p5_256.json" > "$OUT/3d_p5_256.log" 2>&1 || exit 1
run --ndim 3 --cells 256 --p 5 --reps 10 --rounds 2 --variants 0,4,7,9 --kinds apply,jacobi --flush --json "$OUT/3d_p5_256_variants.json" > "$OUT/3d_p5_256_variants.log" 2>&1 || exit 1
run --ndim 3 --cells 512 --p 3 --reps 10 --rounds 2 --kinds apply,residual,jacobi,dot --json "$OUT/3d_p3_512.json" > "$OUT/3d_p3_512.log" 2>&1 || exit 1
echo configs done
