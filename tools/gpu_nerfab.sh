#!/bin/bash
# NeRF-side change check: parity tests touching the marchers, then C3 A/B and a thin-band timeline.
export TMPDIR=/tmp
mkdir -p gpurun_out/nerfab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bands.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/nerfab/pytest.log 2>&1 || { tail -30 gpurun_out/nerfab/pytest.log; exit 1; }
tail -2 gpurun_out/nerfab/pytest.log
bash tools/gpu_c3ab.sh ";" || exit 1
bash tools/gpu_c3ab_serial.sh ";" || exit 1
timeout -k 10 200 python tools/small_band.py 463 521 serial 2>&1 | grep -v amdgpu.ids
