#!/bin/bash
# Serialized-stream stage times + per-kernel table (rocprofv3 kernel trace) for config c3.
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp
timeout -k 10 300 python tools/diag.py > gpurun_out/diag.log 2>&1; rc=$?; echo "diag rc=$rc"; grep -v amdgpu.ids gpurun_out/diag.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --serial-streams > gpurun_out/prof2/stdout.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/prof2 -name '*kernel_trace.csv' | head -1)
python tools/kernel_table.py "$f" generate_kernel 60 > gpurun_out/prof2/table.txt; cat gpurun_out/prof2/table.txt
