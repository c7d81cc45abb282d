set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "msr or bands or onestep" > $O/test.log 2>&1; rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-sweep --config c4 > $O/c4.log 2>&1 && echo "c4 $(grep -o '"value": [0-9.]*' $O/c4.log | head -1) $(grep -o 'rounds_per_frame": [0-9]*' $O/c4.log | tail -1)" || exit 1
for n in 2 4 8; do timeout -k 10 600 python3 -u tools/band8.py --n $n --config c4 --out $O/band_split_c4.jsonl > $O/band8_$n.log 2>&1 || exit 1; done
grep -o '"n": [0-9]*\|"pred_eff": [0-9.]*\|"max_band_ms": [0-9.]*\|"full_ms": [0-9.]*\|"full_msr_rounds": [0-9]*' $O/band_split_c4.jsonl | paste - - - - - 
