#!/bin/bash
# Round-5 first session: A/B of the Jacobi regression fix (round-4 v5 vs the gated
# zeroed rings), the effective clock of the p = 3 kernels, SQ counters of the kept
# Jacobi / apply builds, then the GPU suite, smoke, benches and a 3D kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
O=gpurun_out/${1:-r05s1}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
for rnd in 1 2; do
  for L in main poms_amd/exp/lib_zr.so poms_amd/exp/lib_r04.so; do
    tag=$(basename $L .so); lib=$R/poms_amd/libpoms_hip.so; [ "$L" = main ] || lib=$R/$L
    POMS_HIP_LIB=$lib timeout -k 10 200 python tools/kernel_bench.py --reps 40 --rounds 2 --kinds apply,jacobi,from_zero \
        > $O/kb_${tag}_$rnd.log 2>&1; rc=$?; echo "kb $tag $rnd rc=$rc"; [ $rc -eq 0 ] || stop kb $rc
    grep -o '"kind": "[a-z_]*", "median_us": [0-9.]*' $O/kb_${tag}_$rnd.log | sed "s/^/$tag r$rnd /"
  done
done
timeout -k 10 200 python tools/v5_stamps.py --kinds apply,jacobi --reps 4 --json $O/stamps.json > $O/stamps.log 2>&1; rc=$?
echo "stamps rc=$rc"; cut -c1-400 $O/stamps.log | tail -8; [ $rc -eq 0 ] || stop stamps $rc
for sk in 0 2 6; do   # Jacobi HBM traffic with odd tile rows started late (POMS_V5_SKEW, ~1 us per unit)
  POMS_V5_SKEW=$sk bash tools/pmc_traffic.sh r05_jac_sk$sk kron_v5 --kinds jacobi > $O/pmct_sk$sk.log 2>&1; rc=$?
  echo "pmct skew=$sk rc=$rc $(tail -1 $O/pmct_sk$sk.log | cut -c1-300)"; [ $rc -eq 0 ] || stop pmct $rc
done
for sk in 0 2 6 0 2 6; do
  POMS_V5_SKEW=$sk timeout -k 10 200 python tools/kernel_bench.py --reps 30 --rounds 2 --kinds apply,jacobi > $O/kb_sk$sk.log 2>&1; rc=$?
  echo "kb skew=$sk $(grep -o '"kind": "[a-z_]*", "median_us": [0-9.]*' $O/kb_sk$sk.log | tr '\n' ' ')"; [ $rc -eq 0 ] || stop kb_sk $rc
done
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/$O/clock -o clk -- \
    python3 $R/tools/kernel_bench.py --rounds 1 --reps 20 --kinds apply,jacobi,from_zero) > $O/clock.log 2>&1
rc=$?; echo "clock rc=$rc"; [ $rc -eq 0 ] || stop clock $rc
python3 tools/clock_summary.py $O/clock kron_v5 | tee $O/clock_summary.txt
bash tools/pmc_sq.sh r05jac --kinds apply,jacobi > $O/pmc_sq.log 2>&1; rc=$?; echo "pmc_sq rc=$rc"; [ $rc -eq 0 ] || stop pmc_sq $rc
python3 tools/pmc_summary.py gpurun_out/pmc_r05jac kron_v5 > $O/pmc_sq_summary.txt; cat $O/pmc_sq_summary.txt | head -40
echo "s1 done"
