#!/bin/bash
# Round-5 session 6: kernel traces of the exchange micro-benchmark and of the loopback
# proxy with RCCL and with the peer transport.
set -o pipefail
O=gpurun_out/s6
R=$GRAFT_REPO_ROOT
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/pb -o pb -- python3 $R/tools/r05/peer_bench.py --reps 20 > $R/$O/peer_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/rccl -o proxy -- python3 $R/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $R/$O/proxy_rccl.log 2>&1 || exit 2
POMS_COMM_PEER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/peer -o proxy -- python3 $R/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 > $R/$O/proxy_peer.log 2>&1 || exit 3
echo done
