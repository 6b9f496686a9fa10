set -u
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_v6.py -x -v --timeout 120 --timeout-method thread > $O/pt_v6.log 2>&1; tail -4 $O/pt_v6.log
for L in base allfast2 nostore; do
  POMS_HIP_LIB=$PWD/poms_amd/exp/libv6_$L.so timeout -k 10 200 python tools/kernel_bench.py --cells 512 --p 3 --reps 10 --rounds 2 --variants 10,11 --kinds apply 2>&1 | grep -v amdgpu.ids | sed "s/^/$L /" >> $O/kb.log || exit 1
done
cat $O/kb.log
