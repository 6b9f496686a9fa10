set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/kb_p5.log
for P in 5 4; do
timeout -k 10 300 python tools/kernel_bench.py --cells 256 --p $P --reps 10 --rounds 2 --kinds apply,jacobi,residual --variants 7,9,10 --flush >> gpurun_out/kb_p5.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --p 5 --cells 256 --steps 3 --warmup 1 --no-cpu-baseline --pmc-json "" > gpurun_out/bench_p5.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --p 2 --cells 256 --steps 3 --warmup 1 --no-cpu-baseline --pmc-json "" > gpurun_out/bench_p2.log 2>&1 || exit 1
