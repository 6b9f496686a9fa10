#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/ubofs; mkdir -p $O
timeout -k 10 300 python -u tools/r06/ublib_offsets.py -1 > $O/times.log 2>&1; rc=$?; tail -1 $O/times.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp
for c in 0 1 2 3 4 5 6 7; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/c${c}_$grp -o pmc -- python3 $GRAFT_REPO_ROOT/tools/r06/ublib_offsets.py $c > $O/c${c}_$grp.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "pmc $c $grp rc=$rc"; exit $rc; }
  done
done
python3 - <<'PY'
import csv, glob, os
O=os.environ['GRAFT_REPO_ROOT']+'/gpurun_out/ubofs'
dof=515**3
for c in range(8):
    out=[]
    for g in ('FETCH_SIZE','WRITE_SIZE'):
        v=[float(r['Counter_Value']) for f in glob.glob(f'{O}/c{c}_{g}/**/*counter_collection.csv', recursive=True)
           for r in csv.DictReader(open(f)) if r['Counter_Name']==g and 't16_k' in r['Kernel_Name']]
        m=sum(v)/len(v)*1024*(2 if g=='FETCH_SIZE' else 1) if v else float('nan')
        out.append(m/dof)
    print(f'config {c}: read {out[0]:.2f} write {out[1]:.2f} B/DOF')
PY
