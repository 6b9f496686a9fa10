#!/bin/bash
# Round-5 session 14: the gated launch's exchange kernel under contention -- more
# exchange workgroups.
set -o pipefail
O=gpurun_out/s14
mkdir -p $O
export PYTHONUNBUFFERED=1
for g in 64 128 256; do
  POMS_COMM_PEER=1 POMS_PEER_GATED=1 POMS_PEER_WGS=$g timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_gated_g$g.log 2>&1 || exit 1
  POMS_COMM_PEER=1 POMS_PEER_WGS=$g timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_peer_g$g.log 2>&1 || exit 2
done
echo done
