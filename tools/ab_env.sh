#!/usr/bin/env bash
# Interleaved A/B of one command under several environment settings on one GPU box
# (the pool's boxes differ by several per cent, so a comparison runs on one box, the
# settings alternating).  Each run is its own process under its own time limit; the
# first failure ends the session.  Prints the run's last "ms_per_step" / "median_us"
# / "ms_per_cycle" figures.
#
#   tools/ab_env.sh <tag> <rounds> "<command>" "<env A>" "<env B>" ...
#
# e.g. the round-6 A/Bs:
#   tools/ab_env.sh j2fz 3 "python bench.py --ndim 2 --no-cpu-baseline" "POMS_J2FZ=1" "POMS_J2FZ=0"
#   tools/ab_env.sh fold 3 "python bench.py --ndim 2 --no-cpu-baseline" "POMS_ALPHA_FOLD=1" "POMS_ALPHA_FOLD=0"
#   tools/ab_env.sh r2d 1 "python bench.py --ndim 2 --no-cpu-baseline" "POMS_V3_2D_R=2" "POMS_V3_2D_R=5"
#   tools/ab_env.sh libs 2 "python bench.py --no-cpu-baseline" "POMS_HIP_LIB=$PWD/ab/a.so" "POMS_HIP_LIB=$PWD/ab/b.so"
#   tools/ab_env.sh xch 2 "python tools/slab_proxy.py --loopback-rank 1 --world 8" "X=0" "NCCL_MAX_P2P_NCHANNELS=8"
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
tag=$1; rounds=$2; cmd=$3; shift 3
O=gpurun_out/ab_$tag; mkdir -p "$O"
limit=${AB_LIMIT:-300}
for r in $(seq 1 "$rounds"); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    log=$O/run_${i}_$r.log
    env $e timeout -k 10 "$limit" $cmd > "$log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "[$e] round $r rc=$rc"; tail -3 "$log"; exit $rc; }
    echo "[$e] round $r: $(grep -o '"\(ms_per_step\|median_us\|ms_per_cycle\)": [0-9.]*' "$log" | tail -3 | tr '\n' ' ')"
  done
done
