#!/bin/bash
# One GPU session on the gpurun box, steps chained so that the first failure ends it
# (each GPU step under its own time limit; no step is retried).  Replaces the
# per-session scripts of rounds 2-3 (tools/r0x_*.sh, git history has them).
#
# Usage: tools/session.sh <tag> <step> [<step> ...]
#   tests            whole GPU suite            smoke     __graft_entry__.smoke()
#   pytest:<paths>   those test files (comma-separated)
#   bench            3D headline bench          bench2d   --ndim 2 bench
#   bench:<args>     bench.py with args (commas for spaces)
#   prof             rocprofv3 --kernel-trace --stats of a 2-cycle 3D bench
#   prof2d           the same for the 2D bench
#   kb:<args>        tools/kernel_bench.py with args (commas for spaces)
#   py:<script,args> any python script with args (commas for spaces)
#   proxy            loopback proxy of rank 1 of 8 (tools/slab_proxy.py)
#   pmc:<tag>:<kernel>:<kb args>   HBM traffic passes (tools/pmc_traffic.sh)
# Output under gpurun_out/<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
R=$(pwd)
tag=$1; shift
O=gpurun_out/$tag; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
run() {  # name limit cmd...
    local name=$1 lim=$2; shift 2
    timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-240
    [ $rc -eq 0 ] || stop "$name" $rc
}
i=0
for step in "$@"; do
    i=$((i + 1))
    case "$step" in
        tests) run pytest_gpu 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf ;;
        pytest:*) a=${step#pytest:}; run pytest_$i 900 python -u -m pytest ${a//,/ } -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -rf ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 600 python bench.py ;;
        bench2d) run bench_2d 300 python bench.py --ndim 2 --no-cpu-baseline ;;
        bench:*) a=${step#bench:}; run bench_$i 600 python bench.py ${a//,/ } ;;
        kb:*) a=${step#kb:}; run kb_$i 600 python tools/kernel_bench.py ${a//,/ } ;;
        py:*) a=${step#py:}; run py_$i 600 python ${a//,/ } ;;
        proxy) run proxy_loop_r1 300 python tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 5 ;;
        prof) (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- \
                  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline) > $O/prof.log 2>&1
              rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || stop prof $rc ;;
        prof2d) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof2d -o run -- \
                  python3 $R/bench.py --ndim 2 --steps 10 --warmup 3 --no-cpu-baseline) > $O/prof2d.log 2>&1
              rc=$?; echo "prof2d rc=$rc"; [ $rc -eq 0 ] || stop prof2d $rc ;;
        pmc:*) IFS=: read -r _ ptag kern kargs <<< "$step"
               run pmc_$ptag 600 bash tools/pmc_traffic.sh $ptag "$kern" ${kargs//,/ } ;;
        *) stop "unknown step $step" 2 ;;
    esac
done
echo "session done"
