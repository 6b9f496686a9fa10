#!/bin/bash
# Round-5 session 8: axis-0 chunk of the split launches on the loopback proxy (auto
# picks 3 chunks of 20 planes for the 59-plane interior) for RCCL, peer-cs, peer-fused;
# and the halo-free 67-plane slab at the same chunks.
set -o pipefail
O=gpurun_out/s8
mkdir -p $O
export PYTHONUNBUFFERED=1
for ch in 0 30 65; do
  timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 --chunk $ch > $O/proxy_rccl_c$ch.log 2>&1 || exit 1
  POMS_COMM_PEER=1 POMS_PEER_FUSED=0 timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 --chunk $ch > $O/proxy_peercs_c$ch.log 2>&1 || exit 2
  POMS_COMM_PEER=1 timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 --chunk $ch > $O/proxy_peer_c$ch.log 2>&1 || exit 3
  timeout -k 10 240 python -u tools/slab_proxy.py --planes 67 --steps 3 --chunk $ch > $O/proxy_planes67_c$ch.log 2>&1 || exit 4
done
echo done
