#!/bin/bash
# C3 A/B, serialized streams (the fused tail alone on the GPU): tools/gpu_c3ab_serial.sh "k=v,k=v;k=v"
export TMPDIR=/tmp
IFS=';' read -ra CASES <<< "$1"
for c in "${CASES[@]}"; do
  sets=""; IFS=',' read -ra KV <<< "$c"; for kv in "${KV[@]}"; do [ -n "$kv" ] && sets="$sets --set $kv"; done
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep --serial-streams $sets > gpurun_out/c3abs.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c3abs.json'));t=d['roofline']['fused_tail'];print('[$c]', 'fps', d['value'], 'tail ms/frame', round(t['ms']/20,3), 'frac', t['frac'], d['stages_ms_last_frame'])"
done
