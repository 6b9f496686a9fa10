set -u
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/l2b
mkdir -p $OUT
cd /tmp
for ch in 515 172 0; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $OUT/c$ch -o pmc -- python3 $GRAFT_REPO_ROOT/tools/kernel_bench.py --rounds 1 --reps 3 --cells 512 --p 3 --kinds apply --variants 101 --chunks $ch > $OUT/c$ch.log 2>&1 || exit 1
done
POMS_TILE_ORDER=1 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $OUT/o1 -o pmc -- python3 $GRAFT_REPO_ROOT/tools/kernel_bench.py --rounds 1 --reps 3 --cells 512 --p 3 --kinds apply --variants 101 --chunks 515 > $OUT/o1.log 2>&1
