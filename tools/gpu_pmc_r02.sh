#!/bin/bash
# Round-2 PMC passes of the bench line (serialized streams): FETCH_SIZE, WRITE_SIZE, MFMA -- each its own
# rocprofv3 run, kernel trace only -- then tools/pmc_summary.py -> profiles/pmc_traffic_r02_<config>.json
# (bench.py reads the network kernel's traffic from it).  usage: tools/gpu_pmc_r02.sh [c3|c4]
set -o pipefail
cfg=${1:-c3}
export TMPDIR=/tmp
d=gpurun_out/pmc_$cfg
mkdir -p $d
args="--config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-sweep --serial-streams"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c -d $d/$c -o run --output-format csv -- python3 bench.py $args > $d/$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -20 $d/$c.log; exit $rc; }
done
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE -d $d/MFMA -o run --output-format csv -- python3 bench.py $args > $d/MFMA.log 2>&1
rc=$?; echo "MFMA rc=$rc"; [ $rc -ne 0 ] && { tail -20 $d/MFMA.log; exit $rc; }
mkdir -p gpurun_out/profiles
python3 tools/pmc_summary.py $d gpurun_out/profiles/pmc_traffic_r02_$cfg.json $cfg
