#!/bin/bash
# Round-5 session 9: graph capture of the distributed smoother with the peer transport
# (the RCCL P2P capture crashed, round-4 verdict item 2), then the loopback proxy with
# the captured speculative smoother.
set -o pipefail
O=gpurun_out/s9
mkdir -p $O
export PYTHONUNBUFFERED=1
POMS_COMM_PEER=1 timeout -k 10 600 python -u tools/graph_rccl_probe.py > $O/graph_probe_peer.log 2>&1; echo "probe rc=$?" >> $O/graph_probe_peer.log
for mode in "0 0" "1 0" "1 2"; do
  set -- $mode
  POMS_COMM_PEER=1 POMS_PCG_SPEC=$1 POMS_PCG_GRAPH=$2 timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_peer_spec$1_graph$2.log 2>&1 || exit 2
done
echo done
