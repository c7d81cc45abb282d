#!/bin/bash
# one-step regime: parity tests (wavefront vs regime, bands, RCCL world 1), then C4 and C3 bench lines
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest_os 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "${PYTEST_K:-onestep or kitchen or fused or mid_frame or rccl}"
run bench_c4 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline
run bench_c3 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
