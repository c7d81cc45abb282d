#!/bin/bash
# raytracer parity tests, cost attribution and a serialized kernel profile
mkdir -p gpurun_out/prof3
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "wavefront or full_frame or band" > gpurun_out/pytest_rt.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_rt.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/rt_diag.py > gpurun_out/rt_diag.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/rt_diag.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --serial-streams > gpurun_out/prof3/stdout.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/prof3 -name '*kernel_trace.csv' | head -1)
python tools/kernel_table.py "$f" > gpurun_out/prof3/table.txt; head -25 gpurun_out/prof3/table.txt; tail -1 gpurun_out/prof3/stdout.log | cut -c1-400
