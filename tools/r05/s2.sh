#!/bin/bash
# Round-5 session 2: the hipGraph + RCCL-loopback probe (stages in child processes),
# then the GPU suite, smoke, both benches and 3D / 2D kernel traces.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
O=gpurun_out/${1:-r05s2}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
timeout -k 10 600 python -u tools/graph_rccl_probe.py > $O/graph_probe.log 2>&1; rc=$?
echo "graph probe rc=$rc"; grep "=== stage" $O/graph_probe.log
[ "${2:-}" = "probe" ] && exit $rc
bash tools/session.sh ${1:-r05s2} tests smoke bench bench2d prof prof2d
