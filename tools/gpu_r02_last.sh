#!/bin/bash
# last round-2 call: full GPU suite + smoke, C2 line, serialized rocprofv3 stats
export TMPDIR=/tmp
bash tools/gpu_r02_final2.sh; rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
mkdir -p gpurun_out/last
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-sweep > gpurun_out/last/bench_c2.log 2>&1 || exit 1
tail -1 gpurun_out/last/bench_c2.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/last/prof_c3s -o c3s --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep --serial-streams > gpurun_out/last/prof_c3s.log 2>&1 || exit 1
echo done
