#!/bin/bash
# network / encoder change check: encode + network parity tests, then C2 / C3 / C3-serialized lines under library variants
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lego.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/netab.log 2>&1; tail -2 gpurun_out/netab.log
for v in ${VARIANTS:-_build}; do
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 python bench.py --config c2 --steps 40 --warmup 5 --no-cpu-baseline --no-sweep > gpurun_out/n2.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/n2.json'));print('$v c2', d['value'], 'net frac', d['roofline']['frac'], 'tail frac', d['roofline'].get('fused_tail',{}).get('frac'))"
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep > gpurun_out/n3.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/n3.json'));print('$v c3', d['value'], 'net frac', d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep --serial-streams > gpurun_out/n3s.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/n3s.json'));t=d['roofline']['fused_tail'];print('$v c3 serial', d['value'], 'tail ms', round(t['ms']/20,3), 'frac', t['frac'])"
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-sweep --serial-streams > gpurun_out/n4.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/n4.json'));print('$v c4 serial', d['value'], 'net frac', d['roofline']['frac'], d['stages_ms_last_frame'])"
done
