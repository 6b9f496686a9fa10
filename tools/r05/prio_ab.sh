set -u
O=gpurun_out/s33; mkdir -p $O
for r in 1 2; do
  for m in 0 1 2; do
    POMS_V5_PRIO=$m timeout -k 10 200 python tools/kernel_bench.py --kinds apply,jacobi,from_zero --rounds 2 --reps 15 > $O/kb_p${m}_$r.log 2>&1 || exit 1
    echo "prio $m $r: $(grep -h median_us $O/kb_p${m}_$r.log | python -c 'import sys,json; print([(d["kind"], round(d["median_us"],1), round(d["min_us"],1)) for d in map(json.loads, sys.stdin)])')"
  done
done
