# A/B of libsng_hip.so variants on the default bench line: tools/gpu_ab.sh "_build _build_x ..." [test-variant]
export TMPDIR=/tmp
for v in $1 $1; do
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$v', 'fps', d['value'], 'frac', r['frac'], 'net_ms', r['avg_launch_ms'])"
done
if [ -n "$2" ]; then
  SNG_LIB_PATH=synerfgine_amd/$2/libsng_hip.so timeout -k 10 500 python -u -m pytest tests/ -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ab_pytest.log; exit $rc
fi
