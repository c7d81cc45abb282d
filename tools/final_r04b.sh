set -o pipefail
O=gpurun_out/r04final2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u bench.py > $O/driver.log 2>&1; rc=$?; grep -o '"value": [0-9.]*' $O/driver.log | head -1; exit $rc
