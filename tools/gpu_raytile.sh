#!/bin/bash
# NeRF ray order A/B (nerf_ray_tile) on the C3 bench line (serialized streams: uncontended network launch)
export TMPDIR=/tmp
for set in "nerf_ray_tile=0" "nerf_ray_tile=8" "nerf_ray_tile=16" "nerf_ray_tile=32"; do
  for cfg in c3 c4; do
    timeout -k 10 200 python bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-sweep --serial-streams --set $set > gpurun_out/rt.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/rt.json'));r=d['roofline'];print('$cfg $set', 'fps', d['value'], 'net frac', r['frac'], 'ms', r['avg_launch_ms'], 'stages', d['stages_ms_last_frame'])"
  done
done
