#!/bin/bash
# kernel averages of one thin band (serialized) under library variants: VARIANTS="_build _build_x" tools/gpu_band_variants.sh r0 r1
export TMPDIR=/tmp
for v in ${VARIANTS:-_build}; do
  SNG_LIB_PATH=synerfgine_amd/$v/libsng_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/bv_$v -o run --output-format csv -- python3 tools/small_band.py ${1:-463} ${2:-521} serial > gpurun_out/bv_$v.log 2>&1 || exit 1
  python3 -c "
import csv
rows = sorted(csv.DictReader(open('gpurun_out/bv_$v/run_kernel_stats.csv')), key=lambda r: -float(r['TotalDurationNs']))
print('$v', ' | '.join(r['Name'].split('(')[0].replace('void ','').replace('sng::','')[:28] + ' ' + str(round(float(r['AverageNs'])/1e3,1)) for r in rows[:9]))"
done
