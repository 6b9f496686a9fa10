#!/bin/bash
# Round 6: peer / RCCL capture tests, then the loopback proxy (rank 1 of 8) with the
# step-by-step smoother loop and with the speculative loop replayed from graphs, over
# RCCL (now capturable) and the peer transport, alternating.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/proxy_graph; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 120 --timeout-method thread > $O/pytest_peer.log 2>&1
rc=$?; tail -5 $O/pytest_peer.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for m in step graph; do
    for tr in rccl peer; do
      if [ $m = graph ]; then export POMS_PCG_SPEC=1 POMS_PCG_GRAPH=2; else export POMS_PCG_SPEC=0 POMS_PCG_GRAPH=0; fi
      if [ $tr = peer ]; then export POMS_COMM_PEER=1; else export POMS_COMM_PEER=0; fi
      timeout -k 10 300 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 5 > $O/proxy_${m}_${tr}_$r.log 2>&1
      rc=$?; echo "$m $tr $r rc=$rc: $(tail -1 $O/proxy_${m}_${tr}_$r.log | cut -c1-220)"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
