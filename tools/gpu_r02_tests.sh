#!/bin/bash
# GPU suite + the snapshot-resume test alone (prints its update differences)
mkdir -p gpurun_out/r02t
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r02t/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r02t/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_snapshot.py -q -s --timeout 200 --timeout-method thread > gpurun_out/r02t/snapshot.log 2>&1
grep -E "resume|passed|failed" gpurun_out/r02t/snapshot.log
