#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ublib; mkdir -p $O
timeout -k 10 300 python -u tools/r06/ublib_bench.py > $O/t.log 2>&1; rc=$?; grep kind $O/t.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$grp -o pmc -- python3 $GRAFT_REPO_ROOT/tools/r06/ublib_bench.py > $O/pmc_$grp.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc $grp rc=$rc"; exit $rc; }
done
python3 - <<'PY'
import csv, glob, os, collections
O=os.environ['GRAFT_REPO_ROOT']+'/gpurun_out/ublib'
dof=515**3
acc=collections.defaultdict(list)
for g in ('FETCH_SIZE','WRITE_SIZE'):
    for f in glob.glob(f'{O}/pmc_{g}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name']==g: acc[(r['Kernel_Name'][:40],g)].append(float(r['Counter_Value']))
for (k,g),v in sorted(acc.items()):
    m=sum(v)/len(v)*1024*(2 if g=='FETCH_SIZE' else 1)
    print(f'{k:40s} {g}: {m/dof:.2f} B/DOF ({len(v)} dispatches)')
PY
