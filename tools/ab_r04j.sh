set -o pipefail
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "msr or bands or onestep or spec" > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
B="python3 -u bench.py --no-cpu-baseline --no-sweep --config c4"
timeout -k 10 300 $B > $O/c4_new.log 2>&1 && echo "new $(grep -o '"value": [0-9.]*' $O/c4_new.log | head -1) $(grep -o 'rounds_per_frame": [0-9]*' $O/c4_new.log | tail -1) $(grep -o '"discarded_frac": [0-9.]*' $O/c4_new.log | tail -1)" &&
SNG_LIB_PATH=synerfgine_amd/_build_old/libsng_hip.so timeout -k 10 300 $B > $O/c4_old.log 2>&1 && echo "old $(grep -o '"value": [0-9.]*' $O/c4_old.log | head -1) $(grep -o 'rounds_per_frame": [0-9]*' $O/c4_old.log | tail -1)" &&
timeout -k 10 300 $B > $O/c4_new2.log 2>&1 && echo "new $(grep -o '"value": [0-9.]*' $O/c4_new2.log | head -1)" &&
timeout -k 10 600 python3 -u tools/band8.py --n 8 --config c4 > $O/band8.log 2>&1; rc=$?
grep -o '"pred_eff": [0-9.]*\|"max_band_ms": [0-9.]*\|"full_ms": [0-9.]*\|"full_msr_rounds": [0-9]*' $O/band8.log | paste - - - - - ; exit $rc
