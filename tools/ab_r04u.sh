set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
for v in "rt_prio2_frac=0" "rt_prio2_frac=0.25" "rt_prio2_frac=0" "rt_prio2_frac=0.25" "rt_prio2_frac=0" "rt_prio2_frac=0.25" "rt_prio2_frac=0" "rt_prio2_frac=0.25"; do
  sets=""; for kv in ${v//+/ }; do sets="$sets --set $kv"; done
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-sweep --config c3 $sets > $O/c3.log 2>&1 || exit 1
  echo "$v $(grep -o '"value": [0-9.]*' $O/c3.log | head -1) $(grep -o '"raytrace": [0-9.]*' $O/c3.log | head -1)"
done
