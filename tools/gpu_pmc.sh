#!/bin/bash
# HBM traffic of the hot kernels: two separate PMC passes (FETCH_SIZE, WRITE_SIZE), kernel trace only,
# then tools/pmc_summary.py -> profiles/pmc_network_r01.json.  Run from the repo root on the GPU box.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c -d gpurun_out/pmc/$c -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --serial-streams > gpurun_out/pmc/$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/pmc/$c.log; exit $rc; }
done
# MFMA utilisation of the same launches: one SQ pass + GRBM_GUI_ACTIVE (counter names from rocprofv3 -L)
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1
grep -o "SQ_[A-Z_0-9]*MFMA[A-Z_0-9]*" gpurun_out/pmc/avail.txt | sort -u | tr '\n' ' '; echo
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE -d gpurun_out/pmc/MFMA -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --serial-streams > gpurun_out/pmc/MFMA.log 2>&1
rc=$?; echo "MFMA rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/pmc/MFMA.log; exit $rc; }
python3 tools/pmc_summary.py gpurun_out/pmc profiles/pmc_network_r01.json && mkdir -p gpurun_out/profiles && cp profiles/pmc_network_r01.json gpurun_out/profiles/
