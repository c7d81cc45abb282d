export TMPDIR=/tmp
for v in ${VARIANTS:-_build}; do
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/v_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sweep --serial-streams > gpurun_out/v_$v.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/v_$v/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('shadow_rays', 'raytrace_kernel', 'init_rays', 'generate_kernel', 'nerf_fused', 'network_kernel')): print('$v', r['Name'][:40], round(float(r['AverageNs'])/1e3,1), 'us')"
done
