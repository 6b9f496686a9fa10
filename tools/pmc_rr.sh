set -u
ROOT="$GRAFT_REPO_ROOT"; OUT="$ROOT/gpurun_out/pmc_rr"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
gi=0
for grp in FETCH_SIZE WRITE_SIZE; do
  gi=$((gi+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d "$OUT/g$gi" -o pmc -- python3 "$ROOT/tools/rr_bench.py" --reps 3 --cycles 0 > "$OUT/g$gi.log" 2>&1
  rc=$?; echo "group $gi rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for k in "mrestrict_kernel<12, 74>" "restrict_pass_kernel<16>" "prolong_pass_kernel<16>" "kron_v5_kernel<3, 1,"; do
  python3 "$ROOT/tools/pmc_traffic.py" "$OUT" "$k" 136590875 "$OUT/traffic_$(echo $k | tr -c 'a-z0-9' '_').json" > /dev/null && cat "$OUT/traffic_$(echo $k | tr -c 'a-z0-9' '_').json"; echo
done
