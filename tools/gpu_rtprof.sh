#!/bin/bash
# kernel table of the raytracer under engine overrides: tools/gpu_rtprof.sh "rt_staged=1"
export TMPDIR=/tmp
mkdir -p gpurun_out/rtprof
args=""
for kv in $1; do args="$args --set $kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/rtprof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --serial-streams $args > gpurun_out/rtprof/log 2>&1; echo "rc=$?"
f=$(find gpurun_out/rtprof -name '*kernel_trace.csv' | head -1)
python3 tools/kernel_table.py "$f" rt_ 40 | head -30
