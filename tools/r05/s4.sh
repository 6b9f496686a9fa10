#!/bin/bash
# Round-5 session 4: the peer transport of the ghost exchange (loopback unit tests,
# real neighbours in processes sharing the GPU, then the one-rank loopback proxy
# with RCCL vs the peer kernel).
set -o pipefail
O=gpurun_out/s4
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 120 --timeout-method thread > $O/t_peer.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_dist.py -x -v -m gpu -k "native_schedule or fullsize" --timeout 300 --timeout-method thread > $O/t_dist.log 2>&1 || exit 2
for rep in 1 2; do
  timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_rccl_$rep.log 2>&1 || exit 3
  POMS_COMM_PEER=1 timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_peer_$rep.log 2>&1 || exit 4
done
POMS_COMM_PEER=1 POMS_PEER_WGS=16 timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_peer16.log 2>&1 || exit 5
POMS_COMM_PEER=1 POMS_PEER_WGS=128 timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_peer128.log 2>&1 || exit 6
echo done
