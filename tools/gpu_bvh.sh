#!/bin/bash
# BVH traversal change check: the raytracer parity tests, the C3 line (concurrent), and serialized kernel
# times from rocprofv3.  usage: tools/gpu_bvh.sh [tag]
tag=${1:-bvh}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "full_frame or raytracer or wide_bvh or rt_counting or band_rendering or record_lists" > gpurun_out/$tag/pytest.log 2>&1 || { tail -30 gpurun_out/$tag/pytest.log; exit 1; }
tail -2 gpurun_out/$tag/pytest.log
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep > gpurun_out/$tag/c3.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/$tag/c3.json'));print('c3 fps', d['value'], d['stages_ms_last_frame'], d.get('bvh'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o c3s --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep --serial-streams > gpurun_out/$tag/prof.log 2>&1 || exit 1
f=$(ls gpurun_out/$tag/prof/*/c3s_kernel_stats.csv 2>/dev/null | head -1)
[ -z "$f" ] && f=$(find gpurun_out/$tag/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f"{r['Name'][:70]:70s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.1f} total_ms {float(r['TotalDurationNs'])/1e6:8.2f}")
EOF
