export TMPDIR=/tmp
for v in _build _build_nopow _build_noshade; do
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/v_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sweep --serial-streams > gpurun_out/v_$v.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/v_$v/run_kernel_stats.csv')):
    if 'shadow_rays' in r['Name'] or 'raytrace_kernel' in r['Name'] or 'accumulate' in r['Name']: print('$v', r['Name'][:40], round(float(r['AverageNs'])/1e3,1), 'us')"
done
