#!/bin/bash
# Round 6: memory-only march models (tools/r06/ubench_march2.hip), times and HBM traffic per case.
set -u
cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/ub2
mkdir -p $O
B=$PWD/tools/r06/ubench_march2.bin
FILL=${FILL:-0}
timeout -k 10 120 $B -1 $FILL > $O/times.log 2>&1; rc=$?; cat $O/times.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp
for c in ${CASES:-1 2 3 4 5 6 7}; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_${c}_$grp -o pmc -- $B $c $FILL > $O/pmc_${c}_$grp.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "pmc $c $grp rc=$rc"; exit $rc; }
  done
done
python3 - <<'PY'
import csv, glob, os
O=os.environ.get('GRAFT_REPO_ROOT','.')+'/gpurun_out/ub2'
dof=515**3
for c in range(1,8):
    r={}
    for g in ('FETCH_SIZE','WRITE_SIZE'):
        v=[]
        for f in glob.glob(f'{O}/pmc_{c}_{g}/**/*counter_collection.csv', recursive=True):
            for row in csv.DictReader(open(f)):
                if row['Counter_Name']==g and 'copy' not in row['Kernel_Name']: v.append(float(row['Counter_Value']))
        r[g]=sum(v)/len(v) if v else float('nan')
    rd=2*r['FETCH_SIZE']*1024; wr=r['WRITE_SIZE']*1024
    print(f'case {c}: read {rd/dof:.2f} B/DOF  write {wr/dof:.2f} B/DOF  total {(rd+wr)/dof:.2f}')
PY
