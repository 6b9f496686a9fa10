#!/bin/bash
# Round-5 session 1b: m2 (the 2D row-marching kernel) parity, the 2D sweep and cycle
# A/B against the round-4 2D kernels (POMS_M2=0), m2 row-chunk sweep; the graph probe.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
O=gpurun_out/${1:-r05s1b}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_m2.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_m2.log 2>&1; rc=$?
echo "pytest m2 rc=$rc"; tail -3 $O/pytest_m2.log; [ $rc -eq 0 ] || stop pytest_m2 $rc
for m2 in 0 1; do
  POMS_M2=$m2 timeout -k 10 200 python tools/kernel_bench.py --ndim 2 --cells 1024 --reps 50 --rounds 2 --kinds apply,residual,jacobi,apply_dot \
     --chunks 0 > $O/kb2d_m2$m2.log 2>&1; rc=$?
  echo "kb2d m2=$m2 $(grep -o '"kind": "[a-z_]*", "median_us": [0-9.]*' $O/kb2d_m2$m2.log | tr '\n' ' ')"; [ $rc -eq 0 ] || stop kb2d $rc
done
timeout -k 10 200 python tools/kernel_bench.py --ndim 2 --cells 1024 --reps 50 --rounds 2 --kinds jacobi --chunks 4,8,12,16,24,32 \
     > $O/kb2d_chunks.log 2>&1; rc=$?
echo "kb2d chunks rc=$rc"; grep -o '"chunk": [0-9]*.*"median_us": [0-9.]*' $O/kb2d_chunks.log | sed 's/"tile_cols.*"kind"/ /'; [ $rc -eq 0 ] || stop kb2d_chunks $rc
for r in 1 2; do for m2 in 0 1; do
  POMS_M2=$m2 timeout -k 10 300 python bench.py --ndim 2 --no-cpu-baseline > $O/bench2d_m2${m2}_$r.log 2>&1; rc=$?
  echo "bench2d m2=$m2 r$r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench2d_m2${m2}_$r.log)"; [ $rc -eq 0 ] || stop bench2d $rc
done; done
timeout -k 10 600 python -u tools/graph_rccl_probe.py > $O/graph_probe.log 2>&1; rc=$?
echo "graph probe rc=$rc"; grep -A3 "=== stage" $O/graph_probe.log | cut -c1-300
echo "s1b done"
