#!/bin/bash
# Round-5 session 7: the exchange inside the interior launch (peer transport, fused):
# unit tests, real neighbours, then the loopback proxy (RCCL / peer on the
# communication stream / peer fused) with a kernel trace of the fused one.
set -o pipefail
O=gpurun_out/s7
R=$GRAFT_REPO_ROOT
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -x -q --timeout 120 --timeout-method thread > $O/t_peer.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_dist.py -x -v -m gpu -k "native_schedule or fullsize" --timeout 300 --timeout-method thread > $O/t_dist.log 2>&1 || exit 2
for rep in 1 2; do
  timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_rccl_$rep.log 2>&1 || exit 3
  POMS_COMM_PEER=1 POMS_PEER_FUSED=0 timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_peercs_$rep.log 2>&1 || exit 4
  POMS_COMM_PEER=1 timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_peer_$rep.log 2>&1 || exit 5
done
for g in 16 64; do
  POMS_COMM_PEER=1 POMS_PEER_WGS=$g timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_peer_g$g.log 2>&1 || exit 6
done
cd /tmp && export TMPDIR=/tmp
POMS_COMM_PEER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o proxy -- python3 $R/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $R/$O/prof_peer.log 2>&1 || exit 7
echo done
