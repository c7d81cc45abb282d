#!/bin/bash
# batched cascade loads in occ_step: parity (kitchen/C4 paths, G-buffer) + C4 bench
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest_e 500 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "${PYTEST_K:-kitchen or c4 or gbuffer or onestep or fused or mid_frame}"
run bench_c4 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline --no-sweep --serial-streams
python3 -c "import json;d=json.loads(open('gpurun_out/bench_c4.log').read().strip().splitlines()[-1]);print(d['value'], d['stages_ms_last_frame'])"
