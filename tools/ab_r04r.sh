set -o pipefail
O=gpurun_out/r04r; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || exit $rc
for cfg in c4 c2 c4 c2; do for v in new old; do
  if [ $v = old ]; then export SNG_LIB_PATH=synerfgine_amd/_build_old/libsng_hip.so; else unset SNG_LIB_PATH; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-sweep --config $cfg > $O/${cfg}_$v.log 2>&1 || exit 1
  echo "$cfg $v $(grep -o '"value": [0-9.]*' $O/${cfg}_$v.log | head -1)"
done; done
