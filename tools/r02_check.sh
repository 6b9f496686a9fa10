set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --ndim 2 --steps 5 --warmup 2 > gpurun_out/bench2d.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/slab_proxy.py --planes 67 --steps 3 > gpurun_out/proxy.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/slab_proxy.py --planes 515 --steps 2 > gpurun_out/proxy_full.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_proxy -o proxy -- python -u $GRAFT_REPO_ROOT/tools/slab_proxy.py --planes 67 --steps 3 > $GRAFT_REPO_ROOT/gpurun_out/proxy_prof.log 2>&1
