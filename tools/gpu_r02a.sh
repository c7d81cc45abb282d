#!/bin/bash
# round-2 check: lego views probe, the GPU suite, a bench line (with the new CPU baseline legs)
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run views 200 python tools/lego_views.py
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
run bench 500 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS}
