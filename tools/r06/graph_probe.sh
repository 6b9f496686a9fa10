#!/bin/bash
# Round 6: graph capture of RCCL calls from the C API, one process per stage, with the
# ROCm RCCL (2.27.7) and with torch's bundled RCCL (2.26.6, the one every library run
# loads because torch is imported first).  Usage: graph_probe.sh "lib:stage:mode ..."
# Stops at the first crash, abort or time limit.
# item = lib:stage:mode[:doubles per message[:InitRankConfig 0/1[:buffer offset, doubles]]] (nothing more runs on the GPU then).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/graph_probe; mkdir -p $O
B=$PWD/tools/r06/graph_probe.bin
TL=$(mktemp -d)
TH=$(mktemp -d)
ln -s /usr/local/lib/python3.10/dist-packages/torch/lib/librccl.so $TL/librccl.so.1
# torchhip: torch's bundled HIP 7.0 runtime and HSA runtime as well (what a process that
# imported torch runs on: same SONAMEs, loaded first)
for f in librccl.so:librccl.so.1 libamdhip64.so:libamdhip64.so.7 libhsa-runtime64.so:libhsa-runtime64.so.1; do
  ln -s /usr/local/lib/python3.10/dist-packages/torch/lib/${f%%:*} $TH/${f##*:}
done
for item in $1; do
  IFS=: read lib st mode n cfg off <<< "$item"
  n=${n:-1048576}
  export PROBE_CONFIG=${cfg:-0} PROBE_OFFSET=${off:-0}
  log=$O/${lib}_${st}_${mode}_${n}_c${PROBE_CONFIG}_o${PROBE_OFFSET}.log
  if [ $lib = torch ]; then
    LD_LIBRARY_PATH=$TL:${LD_LIBRARY_PATH:-} timeout -k 5 60 $B $st $mode $n > $log 2>&1
  elif [ $lib = torchhip ]; then
    LD_LIBRARY_PATH=$TH:/usr/local/lib/python3.10/dist-packages/torch/lib:${LD_LIBRARY_PATH:-} timeout -k 5 60 $B $st $mode $n > $log 2>&1
  else
    timeout -k 5 60 $B $st $mode $n > $log 2>&1
  fi
  rc=$?
  echo "=== $lib $st $mode $n config $PROBE_CONFIG offset $PROBE_OFFSET: exit $rc"
  grep -E "RCCL [0-9]|HIP version|captured|FAIL|ok$|values ok|step" $log | tail -5
  case $rc in 124|134|137|139) echo "crash / abort / time limit: stopping"; exit 1;; esac
done
exit 0
