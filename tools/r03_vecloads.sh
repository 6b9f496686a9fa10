#!/bin/bash
# In-cycle A/B of the flat vector kernels' loads: non-temporal (default) vs plain
# (POMS_VEC_LOADS=plain), 3D bench interleaved three times on one box, then a rocprof
# kernel summary of each.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03vecloads; mkdir -p $O
export TMPDIR=/tmp
for rnd in 1 2 3; do for m in nt plain; do
  POMS_VEC_LOADS=$m timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > $O/bench_${m}_r$rnd.log 2>&1 || { echo STOP; exit 1; }
  echo "$m r$rnd $(python3 -c "import json; d=[json.loads(l) for l in open('$O/bench_${m}_r$rnd.log') if l.startswith('{')][-1]; print(round(d['ms_per_step'],2), round(d['roofline']['avg_launch_us'],1))")"
done; done
for m in nt plain; do
  (cd /tmp && POMS_VEC_LOADS=$m timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$m -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline) > $O/prof_$m.log 2>&1 || { echo STOP; exit 1; }
  python3 -c "
import csv
r=list(csv.DictReader(open('$O/prof_$m/run_kernel_stats.csv')))
print('$m', [(x['Name'][:28], round(float(x['AverageNs'])/1e3,1)) for x in r if 'vec_flat' in x['Name']])"
done
