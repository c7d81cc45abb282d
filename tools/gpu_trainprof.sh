# training kernel times (rocprofv3 stats over N steps of tools/train_lego.py) for library variants
export TMPDIR=/tmp
for v in ${VARIANTS:-_build}; do
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tp_$v -o run --output-format csv -- python3 tools/train_lego.py ${STEPS:-300} gpurun_out/t.ingp > gpurun_out/tp_$v.log 2>&1 || exit 1
  grep -i "steps/s\|it/s\|ms/step" gpurun_out/tp_$v.log | tail -2 | cut -c1-200
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/tp_$v/run_kernel_stats.csv')):
    if 'train' in r['Name']: print('$v', r['Name'][:50], round(float(r['AverageNs'])/1e3,1), 'us')"
done
