#!/bin/bash
# GPU suite + C3 and C4 bench lines
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
run bench_c3 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
run bench_c4 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline
