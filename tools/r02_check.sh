set -u
cd $GRAFT_REPO_ROOT
: > gpurun_out/kb_chk.log
for sp in 0 1 2 0; do
POMS_V5_STORE=$sp timeout -k 10 300 python tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 2 --kinds apply,jacobi --variants 10 | sed "s/^{/{\"sp\": $sp, /" >> gpurun_out/kb_chk.log || exit 1
done
POMS_V5_STORE=1 bash tools/pmc_traffic.sh j10sc1 "kron_v5_kernel<3, 2, 3, 0, 18," --cells 512 --p 3 --kinds jacobi --variants 10
POMS_V5_STORE=1 bash tools/pmc_traffic.sh a10sc1 "kron_v5_kernel<3, 0, 4, 0, 26," --cells 512 --p 3 --kinds apply --variants 10
