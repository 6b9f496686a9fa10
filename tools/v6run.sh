set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "11 or 10" -p no:cacheprovider > gpurun_out/pt_v6.log 2>&1; echo rc=$? >> gpurun_out/pt_v6.log
: > gpurun_out/kb_v6.log
kb() { timeout -k 10 200 python tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 2 "$@"; }
for ORD in 0 1; do
  POMS_TILE_ORDER=$ORD kb --kinds apply --variants 10,101,11,111,112 | sed "s/^{/{\"ord\": $ORD, /" >> gpurun_out/kb_v6.log || exit 1
  POMS_TILE_ORDER=$ORD kb --kinds jacobi,residual --variants 10,11 | sed "s/^{/{\"ord\": $ORD, /" >> gpurun_out/kb_v6.log || exit 1
done
POMS_TILE_ORDER=1 POMS_V6_CFG0=8x3 kb --kinds apply --variants 11,111,112 | sed "s/^{/{\"cfg\": \"8x3\", /" >> gpurun_out/kb_v6.log
POMS_TILE_ORDER=1 POMS_V6_CFG0=8x2 kb --kinds apply --variants 11,111,112 | sed "s/^{/{\"cfg\": \"8x2\", /" >> gpurun_out/kb_v6.log
POMS_TILE_ORDER=1 POMS_V6_CFG0=16x1 kb --kinds apply --variants 11,111,112 | sed "s/^{/{\"cfg\": \"16x1\", /" >> gpurun_out/kb_v6.log
