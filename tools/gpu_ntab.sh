#!/bin/bash
# A/B: non-temporal coordinate loads / output stores in nerf_network_kernel (-DNET_NT) vs default
export TMPDIR=/tmp
for v in _build _build_nt _build _build_nt; do
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-sweep > gpurun_out/nt3.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/nt3.json'));print('$v c3', d['value'], 'net frac', d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 python bench.py --config c2 --steps 40 --warmup 5 --no-cpu-baseline --no-sweep > gpurun_out/nt2.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/nt2.json'));print('$v c2', d['value'], 'net frac', d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
done
