#!/bin/bash
# 16-wave v5 two-sweeps-from-zero at p <= 3 + nt loads in the flat vector kernels:
# parity of the touched kernels, then J0 timing v9 (v3) vs v10 (v5) at 515^3 p = 3
# and 256^3 p = 2, then the headline bench.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/j0
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solvers.py -m gpu -x -v --timeout 120 --timeout-method thread -k "from_zero or fused or vec or pcg or vcycle" > $O/pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pt.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 3 --variants 9,10 --kinds from_zero,jacobi > $O/kb_j0_p3.log 2>&1
rc=$?; echo "kb p3 rc=$rc"; tail -4 $O/kb_j0_p3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 3 --variants 10,109 --kinds apply,jacobi > $O/kb_cp.log 2>&1
rc=$?; echo "kb cp rc=$rc"; tail -4 $O/kb_cp.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/kernel_bench.py --cells 256 --p 2 --reps 10 --rounds 3 --variants 9,10 --kinds from_zero > $O/kb_j0_p2.log 2>&1
rc=$?; echo "kb p2 rc=$rc"; tail -2 $O/kb_j0_p2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --kron-reps 5) > $O/prof.log 2>&1
echo "prof rc=$?"
timeout -k 10 300 python -u bench.py --ndim 2 --no-cpu-baseline > $O/bench_2d.log 2>&1
echo "bench2d rc=$?"; tail -1 $O/bench_2d.log | cut -c1-300
export TMPDIR=/tmp
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $ctr | cut -d' ' -f1)
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$GRAFT_REPO_ROOT/$O/pmc_$tag" -o pmc -- \
      python3 "$GRAFT_REPO_ROOT/tools/kernel_bench.py" --rounds 1 --reps 3 --cells 512 --p 3 --kinds jacobi,apply --variants 10) > $O/pmc_$tag.log 2>&1
  echo "pmc $tag rc=$?"
done
