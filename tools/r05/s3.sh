#!/bin/bash
# Round-5 session 3: the loopback proxy of one 8-GPU rank with RCCL's workgroups capped
# (POMS_COMM_CTAS: the exchange kernel beside the interior launch takes fewer CUs), and
# axis-0 chunk sweeps of the p = 5 and p = 2 256^3 kernels.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r05s3}; mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 (rc=$2)"; exit "$2"; }
for r in 1 2; do for c in 0 8 16 32; do
  if [ $c = 0 ]; then unset POMS_COMM_CTAS; else export POMS_COMM_CTAS=$c; fi
  timeout -k 10 300 python tools/slab_proxy.py --loopback-rank 1 --world 8 --steps 5 > $O/proxy_ctas${c}_$r.log 2>&1; rc=$?
  echo "proxy ctas=$c r$r rc=$rc $(grep -o '"ms_per_cycle": [0-9.]*' $O/proxy_ctas${c}_$r.log)"; [ $rc -eq 0 ] || stop proxy $rc
done; done
unset POMS_COMM_CTAS
timeout -k 10 300 python tools/slab_proxy.py --planes 67 --steps 5 > $O/proxy_planes67.log 2>&1; rc=$?
echo "proxy halo-free 67 planes rc=$rc $(grep -o '"ms_per_cycle": [0-9.]*' $O/proxy_planes67.log)"; [ $rc -eq 0 ] || stop proxy67 $rc
for p in 5 2; do
  timeout -k 10 300 python tools/kernel_bench.py --cells 256 --p $p --reps 30 --rounds 2 --kinds apply,jacobi --flush --chunks 0,16,24,32,48,64,96,128 \
      > $O/kb_p${p}_chunks.log 2>&1; rc=$?
  echo "kb p=$p rc=$rc"; grep -o '"chunk": [0-9]*.*"kind": "[a-z]*", "median_us": [0-9.]*' $O/kb_p${p}_chunks.log | sed 's/"tile_cols.*"kind"/ /'; [ $rc -eq 0 ] || stop kb $rc
done
echo "s3 done"
