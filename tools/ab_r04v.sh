set -o pipefail
O=gpurun_out/r04v; mkdir -p $O
for n in 2 4 8; do timeout -k 10 600 python3 -u tools/band8.py --n $n --config c3 --out $O/band_split_c3.jsonl > $O/band8_$n.log 2>&1 || exit 1; done
grep -o '"n": [0-9]*\|"pred_eff": [0-9.]*\|"max_band_ms": [0-9.]*\|"full_ms": [0-9.]*\|"pred_eff_compute_only": [0-9.]*' $O/band_split_c3.jsonl | paste - - - - - - - -
