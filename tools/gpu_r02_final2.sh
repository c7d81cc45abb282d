#!/bin/bash
# closing check: full GPU suite + smoke
mkdir -p gpurun_out/r02f
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r02f/pytest_gpu.log 2>&1
rc=$?; tail -8 gpurun_out/r02f/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02f/smoke.log 2>&1; rc2=$?
tail -3 gpurun_out/r02f/smoke.log; echo "pytest rc=$rc smoke rc=$rc2"
