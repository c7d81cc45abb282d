#!/bin/bash
# C4 generate-grid A/B (nerf_gen_wide, nerf_gen_blocks)
export TMPDIR=/tmp
for set in "nerf_gen_wide=1" "nerf_gen_wide=0" "nerf_gen_blocks=-1" "nerf_gen_wide=0 --set nerf_gen_blocks=-1"; do
  timeout -k 10 200 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --serial-streams --set $set > gpurun_out/gab.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/gab.json'));print('$set', 'fps', d['value'], d['stages_ms_last_frame'])"
done
