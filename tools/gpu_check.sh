#!/bin/bash
# GPU validation run: smoke -> parity tests -> short bench.  Stops on any fault/timeout
# (exit codes other than 0 = ok / 1 = test failures).
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
run smoke 400 python __graft_entry__.py smoke
run pytest_gpu 900 python -m pytest tests -m gpu -q -rf ${PYTEST_K:+-k "$PYTEST_K"}
run bench 400 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS}
