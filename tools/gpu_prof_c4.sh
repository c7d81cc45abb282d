#!/bin/bash
# rocprofv3 kernel trace + stats of the C4 bench (kernel table per frame), serialized streams
mkdir -p gpurun_out/prof_c4
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o c4 --output-format csv -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof_c4/stdout.log 2>&1
echo "rc=$?"
f=$(find gpurun_out/prof_c4 -name "*kernel_stats.csv" | head -1); echo "$f"; head -30 "$f" | cut -c1-200
