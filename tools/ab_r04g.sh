set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
B="python3 -u bench.py --no-cpu-baseline --no-sweep --config c3"
for f in 0.1 0.15 0.2 0.3 0.5 1 0 0.2; do
  timeout -k 10 300 $B --set rt_prio_frac=$f > $O/c3_$f.log 2>&1 || exit 1
  echo "prio $f $(grep -o '"value": [0-9.]*' $O/c3_$f.log | head -1) $(grep -o '"raytrace": [0-9.]*' $O/c3_$f.log | head -1)"
done
