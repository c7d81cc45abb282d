#!/bin/bash
# rocprofv3 kernel trace of a short bench run (no PMC counters here).
mkdir -p gpurun_out/prof
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_stdout.log 2>&1
echo "rc=$?"
find gpurun_out/prof -name "*stats*" | head
