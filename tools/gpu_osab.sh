#!/bin/bash
# C4 one-step horizon A/B
export TMPDIR=/tmp
for set in "nerf_onestep_horizon=10000" "nerf_onestep_horizon=2048" "nerf_onestep_horizon=1024" "nerf_onestep_horizon=512"; do
  timeout -k 10 200 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --serial-streams --set $set > gpurun_out/oab.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/oab.json'));print('$set', 'fps', d['value'], d['stages_ms_last_frame'], d['roofline']['fused_tail']['ms'])"
done
