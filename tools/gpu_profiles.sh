#!/bin/bash
# Round profile set -> profiles/: default bench (concurrent streams) and serialized bench, each under
# rocprofv3 --kernel-trace --stats, plus the two PMC passes for HBM traffic.  Run on the GPU box.
set -o pipefail
export TMPDIR=/tmp
R=${ROUND:-r01}
mkdir -p gpurun_out/pf gpurun_out/profiles
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > gpurun_out/pf/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/pf/$name.log; exit $rc; }
  return 0
}
run pmc 900 bash tools/gpu_pmc.sh
cp profiles/pmc_network_r01.json gpurun_out/profiles/pmc_network_$R.json
run bench_plain 600 python3 bench.py
grep '^{' gpurun_out/pf/bench_plain.log | tail -1 > gpurun_out/profiles/${R}_bench.json
run bench_default 600 rocprofv3 --kernel-trace --stats -d gpurun_out/pf/default -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
run bench_serial 600 rocprofv3 --kernel-trace --stats -d gpurun_out/pf/serial -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --serial-streams
for m in default serial; do
  grep '^{' gpurun_out/pf/bench_$m.log | tail -1 > gpurun_out/profiles/${R}_bench_$m.json
  cp gpurun_out/pf/$m/run_kernel_stats.csv gpurun_out/profiles/${R}_bench_${m}_kernel_stats.csv
  python3 tools/kernel_table.py gpurun_out/pf/$m/run_kernel_trace.csv nerf_network_kernel 60 > gpurun_out/profiles/${R}_bench_${m}_kernel_table.txt
done
python3 - <<PY
import csv, json
for m in ("default", "serial"):
    b = json.load(open(f"gpurun_out/profiles/${R}_bench_{m}.json"))
    rows = [r for r in csv.DictReader(open(f"gpurun_out/profiles/${R}_bench_{m}_kernel_stats.csv")) if "nerf_network_kernel" in r["Name"]]
    avg_us = float(rows[0]["AverageNs"]) / 1e3 if rows else None
    print(m, "fps", b["value"], "roofline avg_launch_ms", b["roofline"]["avg_launch_ms"], "rocprof avg ms", avg_us and avg_us / 1e3, "frac", b["roofline"]["frac"])
PY
