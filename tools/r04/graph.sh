#!/bin/bash
# Speculative smoother call replayed from a captured hipGraph: parity (Python loop /
# step-by-step / speculative / graph capture / graph replay), the 2D cycle and the
# one-slab proxies with graphs off / on (interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r04graph}; mkdir -p $O
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_solvers.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "speculative or native_pcg or damped_jacobi or device_reduction or timing" > $O/pytest_graph.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_graph.log; [ $rc -eq 0 ] || stop pytest $rc
for r in 1 2; do
  for g in 0 1; do
    POMS_PCG_GRAPH=$g timeout -k 10 300 python bench.py --ndim 2 --no-cpu-baseline > $O/bench2d_g${g}_$r.log 2>&1; rc=$?; echo "2d graph=$g rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench2d_g${g}_$r.log)"; [ $rc -eq 0 ] || stop bench2d $rc
  done
done
for g in 0 1; do
  POMS_PCG_GRAPH=$g timeout -k 10 300 python tools/slab_proxy.py --planes 67 --steps 5 > $O/proxy_planes_g$g.log 2>&1; rc=$?; echo "proxy planes graph=$g rc=$rc"; tail -2 $O/proxy_planes_g$g.log | cut -c1-300; [ $rc -eq 0 ] || stop proxy $rc
done
for g in 0 2; do
  POMS_PCG_GRAPH=$g timeout -k 10 300 python tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 5 > $O/proxy_loop_g$g.log 2>&1; rc=$?; echo "proxy loopback graph=$g rc=$rc"; tail -2 $O/proxy_loop_g$g.log | cut -c1-300; [ $rc -eq 0 ] || stop proxy_loop $rc
done
echo "session done"
