#!/bin/bash
# C4 NeRF-shadow pass split: base vs timing-only builds without the BVH walk / without the NeRF march
export TMPDIR=/tmp
for v in _build _build_nobvh _build_nonerf; do
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-sweep --serial-streams > gpurun_out/sh_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sh_$v.json'));print('$v', 'fps', d['value'], d['stages_ms_last_frame'])"
done
