#!/bin/bash
# Round-5 session 5: exchange micro-benchmark (RCCL self-send vs the peer kernel) and
# the loopback proxy with plain (coarse) mailboxes, with a kernel trace.
set -o pipefail
O=gpurun_out/s5
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -x -q --timeout 120 --timeout-method thread > $O/t_peer.log 2>&1 || exit 9
timeout -k 10 300 python -u tools/r05/peer_bench.py > $O/peer_bench.log 2>&1 || exit 1
for rep in 1 2; do
  POMS_COMM_PEER=1 timeout -k 10 240 python -u tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $O/proxy_peer_$rep.log 2>&1 || exit 2
done
cd /tmp && export TMPDIR=/tmp
POMS_COMM_PEER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o proxy_peer -- python3 $GRAFT_REPO_ROOT/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $GRAFT_REPO_ROOT/$O/prof_peer.log 2>&1 || exit 3
echo done
