#!/bin/bash
# C4 A/B of engine parameters: tools/gpu_c4ab.sh "k=v,k=v;k=v" [--serial-streams]
export TMPDIR=/tmp
IFS=';' read -ra CASES <<< "$1"
for c in "${CASES[@]}"; do
  sets=""; IFS=',' read -ra KV <<< "$c"; for kv in "${KV[@]}"; do [ -n "$kv" ] && sets="$sets --set $kv"; done
  timeout -k 10 300 python bench.py --config c4 --steps 4 --warmup 1 --no-cpu-baseline --no-sweep $2 $sets > gpurun_out/c4ab.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c4ab.json'));print('[$c $2]', 'fps', d['value'], d['stages_ms_last_frame'])"
done
