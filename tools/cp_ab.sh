set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cpab; mkdir -p $O
for r in 1 2 3; do
timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 3 --variants 10,104,109 --kinds apply,dot >> $O/kb.log 2>&1 || exit 1
done
grep -h GBps $O/kb.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['variant'], d['kind'], round(d['median_us'],1), round(d['min_us'],1))"
