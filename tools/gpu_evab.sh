#!/bin/bash
# dispatch-recorded network timing events: parity tests of the frame path, bench line and rocprofv3 stats of the same run
export TMPDIR=/tmp
mkdir -p gpurun_out/ev
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lego.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ev/tests.log 2>&1; rc=$?; tail -2 gpurun_out/ev/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/ev/bench.log 2>&1 || exit 1
grep '^{' gpurun_out/ev/bench.log | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('c3', d['value'], 'frac', r['frac'], 'ms', r['avg_launch_ms'], 'psnr', d['psnr_vs_oracle']['db'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ev/prof -o c3 --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep > gpurun_out/ev/prof.log 2>&1 || exit 1
grep '^{' gpurun_out/ev/prof.log | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('c3 under rocprof', d['value'], 'frac', r['frac'], 'ms', r['avg_launch_ms'])"
