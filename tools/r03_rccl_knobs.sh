#!/bin/bash
# Loopback proxy (rank 1 of 8) under RCCL channel knobs: the RCCL kernel's grid and
# time (rocprofv3 kernel trace) and the cycle time, one process per setting.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03knobs}; mkdir -p $O
export TMPDIR=/tmp
for k in "base" "NCCL_MAX_P2P_NCHANNELS=8" "NCCL_NCHANNELS_PER_PEER=2" "NCCL_MAX_NCHANNELS=8" "NCCL_P2P_USE_CUDA_MEMCPY=1"; do
  n=${k%%=*}
  if [ "$k" = base ]; then envs=""; else envs="$k"; fi
  (cd /tmp && env $envs timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$n -o run -- python3 $GRAFT_REPO_ROOT/tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 3 --warmup 1) > $O/proxy_$n.log 2>&1
  rc=$?; echo "$k rc=$rc"; grep '^{' $O/proxy_$n.log | cut -c150-260; [ $rc -eq 0 ] || exit $rc
  python3 - $O/prof_$n/run_kernel_trace.csv <<'PY'
import csv, sys, statistics
r=[x for x in csv.DictReader(open(sys.argv[1])) if 'rccl' in x['Kernel_Name']]
g=set(int(x['Grid_Size_X'])//int(x['Workgroup_Size_X']) for x in r)
d=[(int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e3 for x in r]
print('  rccl kernels', len(r), 'grids', sorted(g), 'median us', round(statistics.median(d),1) if d else None)
PY
done
echo done
