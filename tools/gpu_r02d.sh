#!/bin/bash
# counting-frame test, bench line with the extra legs, PMC passes (C3, C4)
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest_cnt 300 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread -k "counting or snapshot or raytracer"
run bench_c3 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
run pmc_c3 700 bash tools/gpu_pmc_r02.sh c3
run pmc_c4 700 bash tools/gpu_pmc_r02.sh c4
