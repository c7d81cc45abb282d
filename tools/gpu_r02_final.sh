#!/bin/bash
# Round-2 evidence: full GPU suite, smoke, the default bench line (with CPU baselines and the extra legs),
# rocprofv3 kernel stats of the C3 and C4 bench lines
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; date
  timeout -k 10 "$to" "$@" > "gpurun_out/r02/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -3 "gpurun_out/r02/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py
run prof_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02/prof_c3 -o c3 --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep
run prof_c3_serial 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02/prof_c3s -o c3s --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep --serial-streams
run prof_c4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02/prof_c4 -o c4 --output-format csv -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-sweep
