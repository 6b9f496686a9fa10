#!/bin/bash
# Round-5 session 13: the gated distributed launch (v5 MODE 7 beside the peer exchange):
# loopback tests (every epilogue bitwise against RCCL, capture, pcg graph), real
# neighbours, then the loopback proxy: RCCL / peer / peer gated.
set -o pipefail
O=gpurun_out/s13
R=$GRAFT_REPO_ROOT
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 120 --timeout-method thread > $O/t_peer.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_dist.py -x -v -m gpu -k "native_schedule" --timeout 300 --timeout-method thread > $O/t_dist.log 2>&1 || exit 2
for rep in 1 2; do
  timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_rccl_$rep.log 2>&1 || exit 3
  POMS_COMM_PEER=1 timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_peer_$rep.log 2>&1 || exit 4
  POMS_COMM_PEER=1 POMS_PEER_GATED=1 timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_gated_$rep.log 2>&1 || exit 5
done
cd /tmp && export TMPDIR=/tmp
POMS_COMM_PEER=1 POMS_PEER_GATED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o proxy -- python3 $R/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $R/$O/prof_gated.log 2>&1 || exit 6
echo done
