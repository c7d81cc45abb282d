#!/bin/bash
# bench in both stream modes (no cpu baseline) + concurrent-mode kernel profile
export TMPDIR=/tmp
mkdir -p gpurun_out/prof4
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_conc.json 2> gpurun_out/bench_conc.err; rc=$?; echo "conc rc=$rc"; cut -c1-300 gpurun_out/bench_conc.json; python -c "import json;d=json.load(open('gpurun_out/bench_conc.json'));print(d['stages_ms_last_frame'], d['roofline'])"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --serial-streams > gpurun_out/bench_ser.json 2>/dev/null; rc=$?; echo "ser rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/bench_ser.json'));print(d['value'], d['stages_ms_last_frame'], d['roofline'])"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof4/stdout.log 2>&1; rc=$?; echo "prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/prof4 -name '*kernel_trace.csv' | head -1)
python tools/kernel_table.py "$f" nerf_network 40 > gpurun_out/prof4/table.txt; head -12 gpurun_out/prof4/table.txt; tail -2 gpurun_out/prof4/table.txt
