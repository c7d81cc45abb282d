# shadow_rays_kernel time with the BVH half or the NeRF half removed (timing-only builds), plus a
# 2-rank gloo rehearsal of bench.py's band path on the one GPU
export TMPDIR=/tmp
for v in ${VARIANTS:-_build}; do
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ss_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --serial-streams > gpurun_out/ss_$v.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/ss_$v/run_kernel_stats.csv')):
    if 'shadow_rays' in r['Name'] or 'raytrace_kernel' in r['Name']: print('$v', r['Name'][:40], round(float(r['AverageNs'])/1e3,1), 'us')"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --no-cpu-baseline > gpurun_out/gloo2.log 2>&1; rc=$?; grep '^{' gpurun_out/gloo2.log | cut -c1-300; exit $rc
