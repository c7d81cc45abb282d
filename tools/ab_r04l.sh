set -o pipefail
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "megakernel or bands or msr or rt_views or counting or parity" > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/tile_cost.py --config c3 --bounds 501-560 --set rt_tile_h=4 > $O/tile_84.log 2>&1 && grep '^{' $O/tile_84.log
timeout -k 10 900 python3 -u tools/band8.py --n 8 --config c3 --cases "/rt_tile_h=4" > $O/band8_c3.log 2>&1; rc=$?
grep -o '"overrides": {[^}]*}\|"pred_eff": [0-9.]*\|"max_band_ms": [0-9.]*\|"full_ms": [0-9.]*' $O/band8_c3.log | paste - - - - ; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-sweep --config c3 --set rt_tile_h=4 > $O/c3_84.log 2>&1 && echo "c3 8x4 $(grep -o '"value": [0-9.]*' $O/c3_84.log | head -1)"
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-sweep --config c3 > $O/c3.log 2>&1 && echo "c3 8x8 $(grep -o '"value": [0-9.]*' $O/c3.log | head -1)"
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-sweep --config c3 --set rt_colour_in_shadow=0 > $O/c3_nocis.log 2>&1 && echo "c3 colour kernel $(grep -o '"value": [0-9.]*' $O/c3_nocis.log | head -1)"
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-sweep --config c3 > $O/c3b.log 2>&1 && echo "c3 8x8 $(grep -o '"value": [0-9.]*' $O/c3b.log | head -1)"
for b in 16777216 67108864; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-sweep --config c4 --set nerf_msr_budget=$b > $O/c4_$b.log 2>&1 || exit 1
  echo "c4 budget $b $(grep -o '"value": [0-9.]*' $O/c4_$b.log | head -1) $(grep -o 'rounds_per_frame": [0-9]*' $O/c4_$b.log | tail -1) $(grep -o '"discarded_frac": [0-9.]*' $O/c4_$b.log | tail -1)"
done
timeout -k 10 900 python3 -u tools/band8.py --n 8 --config c4 --cases "/nerf_msr_budget=67108864" > $O/band8_c4.log 2>&1; rc=$?
grep -o '"overrides": {[^}]*}\|"pred_eff": [0-9.]*\|"max_band_ms": [0-9.]*\|"full_ms": [0-9.]*' $O/band8_c4.log | paste - - - - ; exit $rc
