#!/bin/bash
# A/B: contiguous per-wave tile runs in nerf_network_kernel (-DNET_CHUNKED) vs the strided walk
export TMPDIR=/tmp
SNG_LIB_PATH=synerfgine_amd/_build_ck/libsng_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "network or nerf_frame or full_frame" --timeout 200 --timeout-method thread > gpurun_out/ck_tests.log 2>&1; rc=$?; tail -1 gpurun_out/ck_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in _build _build_ck _build _build_ck; do
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-sweep > gpurun_out/ck3.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ck3.json'));print('$v c3', d['value'], 'net frac', d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 python bench.py --config c2 --steps 40 --warmup 5 --no-cpu-baseline --no-sweep > gpurun_out/ck2.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ck2.json'));print('$v c2', d['value'], 'net frac', d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
done
