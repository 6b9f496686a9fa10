set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/kernel_bench.py --cells 256 --p 2 --reps 10 --rounds 2 --kinds from_zero,jacobi --variants 10,9 --flush > gpurun_out/kb_chk.log 2>&1
timeout -k 10 200 python tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 2 --kinds apply,jacobi --variants 10 >> gpurun_out/kb_chk.log 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_chk.log 2>&1; echo rc=$? >> gpurun_out/pt_chk.log
