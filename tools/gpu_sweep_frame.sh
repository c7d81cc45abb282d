# full-frame bench under schedule overrides: tools/gpu_sweep_frame.sh "k=v,k=v;k=v" (one line per case)
export TMPDIR=/tmp
IFS=';' read -ra CASES <<< "$1"
for c in "" "${CASES[@]}"; do
  args=""; IFS=',' read -ra KV <<< "$c"; for kv in "${KV[@]}"; do args="$args --set $kv"; done
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline $args > gpurun_out/sweep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sweep.json'));print('[$c]', 'fps', d['value'], 'frac', d['roofline']['frac'])"
done
