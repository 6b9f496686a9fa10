#!/bin/bash
# Round-5 session 10: peer-transport tests (capture of the distributed sweep and the
# pcg graph replay included) and the graph probe's pcg stage with the peer transport.
set -o pipefail
O=gpurun_out/s10
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 120 --timeout-method thread > $O/t_peer.log 2>&1 || exit 1
POMS_COMM_PEER=1 timeout -k 10 300 python -u tools/graph_rccl_probe.py --stages halo,split,pcg > $O/graph_probe_peer.log 2>&1 || exit 2
echo done
