#!/bin/bash
# C3 A/B of engine parameters under a library variant: tools/gpu_c3ab_lib.sh <build dir> "k=v;k=v"
export TMPDIR=/tmp
IFS=';' read -ra CASES <<< "$2"
for c in "${CASES[@]}"; do
  sets=""; IFS=',' read -ra KV <<< "$c"; for kv in "${KV[@]}"; do [ -n "$kv" ] && sets="$sets --set $kv"; done
  SNG_LIB_PATH=synerfgine_amd/$1/libsng_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep $sets > gpurun_out/c3abl.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c3abl.json'));print('[$1 $c]', 'fps', d['value'], d['stages_ms_last_frame'])"
done
