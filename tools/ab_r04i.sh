set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
B="python3 -u bench.py --no-cpu-baseline --no-sweep --config c4"
for b in 16777216 33554432 67108864 16777216; do
  timeout -k 10 300 $B --set nerf_msr_budget=$b > $O/c4_$b.log 2>&1 || exit 1
  echo "budget $b $(grep -o '"value": [0-9.]*' $O/c4_$b.log | head -1) $(grep -o '"msr_rounds": {[^}]*rounds_per_frame": [0-9]*' $O/c4_$b.log | grep -o 'rounds_per_frame": [0-9]*') $(grep -o '"discarded_frac": [0-9.]*' $O/c4_$b.log | tail -1)"
done
timeout -k 10 600 python3 -u tools/band8.py --n 8 --config c4 --cases "/nerf_msr_budget=67108864" > $O/band8.log 2>&1; rc=$?
grep -o '"overrides": {[^}]*}\|"pred_eff": [0-9.]*\|"max_band_ms": [0-9.]*\|"full_ms": [0-9.]*' $O/band8.log | paste - - - - ; exit $rc
