set -o pipefail
mkdir -p gpurun_out/r04f
B="python3 -u bench.py --no-cpu-baseline --no-sweep"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04f/test.log 2>&1 && tail -2 gpurun_out/r04f/test.log &&
SNG_LIB_PATH=synerfgine_amd/_build_old/libsng_hip.so timeout -k 10 300 $B --config c4 > gpurun_out/r04f/c4_old1.log 2>&1 &&
timeout -k 10 300 $B --config c4 > gpurun_out/r04f/c4_new1.log 2>&1 &&
SNG_LIB_PATH=synerfgine_amd/_build_old/libsng_hip.so timeout -k 10 300 $B --config c4 > gpurun_out/r04f/c4_old2.log 2>&1 &&
timeout -k 10 300 $B --config c4 > gpurun_out/r04f/c4_new2.log 2>&1 &&
SNG_LIB_PATH=synerfgine_amd/_build_old/libsng_hip.so timeout -k 10 300 $B --config c3 > gpurun_out/r04f/c3_old1.log 2>&1 &&
timeout -k 10 300 $B --config c3 > gpurun_out/r04f/c3_new1.log 2>&1 &&
timeout -k 10 300 python3 -u tools/tile_cost.py --config c3 --bounds 501-560 --bounds 433-501 --bounds 909-1080 > gpurun_out/r04f/tile_cost.log 2>&1
for f in gpurun_out/r04f/c*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1)"; done; cat gpurun_out/r04f/tile_cost.log | grep '^{'
