set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/l2
mkdir -p $OUT
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for v in 10 101 11 111; do
  kind=apply
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $OUT/v$v -o pmc -- python3 $GRAFT_REPO_ROOT/tools/kernel_bench.py --rounds 1 --reps 3 --cells 512 --p 3 --kinds $kind --variants $v > $OUT/v$v.log 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $OUT/j10 -o pmc -- python3 $GRAFT_REPO_ROOT/tools/kernel_bench.py --rounds 1 --reps 3 --cells 512 --p 3 --kinds jacobi --variants 10 > $OUT/j10.log 2>&1
