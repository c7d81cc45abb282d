set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || exit $rc
B="python3 -u bench.py --no-cpu-baseline --no-sweep --config c4"
for v in new old new old; do
  if [ $v = old ]; then export SNG_LIB_PATH=synerfgine_amd/_build_old/libsng_hip.so; else unset SNG_LIB_PATH; fi
  timeout -k 10 300 $B > $O/c4_$v.log 2>&1 || exit 1
  echo "c4 $v $(grep -o '"value": [0-9.]*' $O/c4_$v.log | head -1)"
done
