#!/bin/bash
# bench sweep over engine overrides: tools/gpu_sweep.sh "rt_start_chunk=0" "rt_start_chunk=1" ...
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
for ov in "$@"; do
  args=""
  for kv in $ov; do args="$args --set $kv"; done
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $args > gpurun_out/sweep/out.json 2>/dev/null; rc=$?
  [ $rc -ne 0 ] && { echo "$ov rc=$rc"; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/sweep/out.json'));r=d['roofline'];print('$ov', 'fps', d['value'], 'frac', r['frac'], 'net_ms', r['avg_launch_ms'], d['stages_ms_last_frame'])"
done
