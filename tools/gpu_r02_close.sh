#!/bin/bash
# Round-2 closing evidence after the per-pixel shutter camera: default bench line, C2 line, rocprofv3 stats (C3 default + serialized)
mkdir -p gpurun_out/r02c
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; date
  timeout -k 10 "$to" "$@" > "gpurun_out/r02c/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -2 "gpurun_out/r02c/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run bench 600 python bench.py
run bench_c2 300 python bench.py --config c2 --no-cpu-baseline --no-sweep
run prof_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02c/prof_c3 -o c3 --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep
run prof_c3_serial 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02c/prof_c3s -o c3s --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep --serial-streams
