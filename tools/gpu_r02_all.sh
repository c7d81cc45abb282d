#!/bin/bash
# one call: GPU suite + snapshot test output, then the closing bench / profiles
bash tools/gpu_r02_tests.sh; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_r02_close.sh
