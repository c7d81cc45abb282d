#!/bin/bash
# C3 A/B of engine parameters (concurrent schedule, the bench default): tools/gpu_c3ab.sh "k=v,k=v;k=v"
export TMPDIR=/tmp
IFS=';' read -ra CASES <<< "$1"
for rep in 1 2; do
for c in "${CASES[@]}"; do
  sets=""; IFS=',' read -ra KV <<< "$c"; for kv in "${KV[@]}"; do [ -n "$kv" ] && sets="$sets --set $kv"; done
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep $sets > gpurun_out/c3ab.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c3ab.json'));print('[$c]', 'fps', d['value'], d['stages_ms_last_frame'])"
done
done
