#!/bin/bash
# tools/gpu.sh -- the one GPU-box runner (replaces the one-off tools/gpu_*.sh scripts of rounds 1-2).
#
# usage (inside gpurun):  TAG=name tools/gpu.sh STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failing step ends the call (no retries).
#   test[:EXPR]            pytest -m gpu over tests/ (-k EXPR when given)
#   bench[:CFG[:ARGS]]     bench.py --config CFG --no-cpu-baseline --no-sweep ARGS   (ARGS: ',' for spaces)
#   driver                 bench.py with no flags (the driver's own line, incl. CPU baseline and extra legs)
#   prof[:CFG[:ARGS]]      rocprofv3 --kernel-trace --stats of a short bench.py run (ARGS as for bench)
#   profdriver             rocprofv3 over bench.py --no-cpu-baseline + tools/roofline_check.py (same-process roofline check)
#   pmc[:CFG[:ARGS]]       FETCH_SIZE / WRITE_SIZE / MFMA PMC passes (one rocprofv3 run each) + tools/pmc_summary.py
#   sq[:CFG[:ARGS]]        SQ_INSTS_* + SQ_WAVE_CYCLES pass with kernel trace + tools/sq_summary.py (VALU roofline)
#   ab:CFG:PAIRS:A/B       PAIRS alternating bench.py runs of two settings (A, B: KEY=V[,KEY=V...], '-' for the defaults),
#                          then tools/bsum.py over the logs (replaces round 4's one-off ab_r04*.sh scripts)
#   abl:CFG:PAIRS:A/B      as ab, but A and B are library builds (synerfgine_amd/_build_A, e.g. make BUILD=_build_x EXTRA=-D...;
#                          '-' for the default _build), loaded with SNG_LIB_PATH
#   sqpy:SCRIPT[:ARGS]     the sq pass over python3 tools/SCRIPT ARGS
#   py:SCRIPT[:ARGS]       python3 tools/SCRIPT ARGS
#   profpy:SCRIPT[:ARGS]   rocprofv3 --kernel-trace --stats of python3 tools/SCRIPT ARGS (+ kernel table)
#   pmcpy:SCRIPT[:ARGS]    FETCH_SIZE / WRITE_SIZE / MFMA passes over python3 tools/SCRIPT ARGS + tools/pmc_summary.py
# Output goes to gpurun_out/$TAG/ (TAG defaults to "run"), one log per step.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  rest=""
  [[ "$step" == *:* ]] && rest=${step#*:}
  cfg=${rest%%:*}
  args=""
  [[ "$rest" == *:* ]] && args=${rest#*:}
  args=${args//,/ }
  log=$OUT/$n.$kind.log
  echo "[gpu.sh] step $n: $step -> $log"
  case $kind in
    test)
      k=()
      [ -n "$rest" ] && k=(-k "$rest")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread "${k[@]}" > $log 2>&1
      rc=$?; tail -5 $log ;;
    bench)
      timeout -k 10 600 python3 -u bench.py --config ${cfg:-c3} --no-cpu-baseline --no-sweep $args > $log 2>&1
      rc=$?; tail -c 3000 $log; echo ;;
    driver)
      timeout -k 10 900 python3 -u bench.py > $log 2>&1
      rc=$?; tail -c 4000 $log; echo ;;
    prof)
      d=$OUT/prof$n
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --config ${cfg:-c3} --steps 10 --warmup 2 --no-cpu-baseline --no-sweep $args > $log 2>&1
      rc=$?
      [ $rc -eq 0 ] && python3 tools/kernel_table.py $(find $d -name "*kernel_trace.csv" | head -1) > $d/kernel_table.txt 2>&1 && head -30 $d/kernel_table.txt ;;
    profdriver)
      # rocprofv3 over the driver-format line without the CPU legs (the serialized leg and the extras run); the
      # roofline fields of that line recomputed from the same process's kernel trace (tools/roofline_check.py)
      d=$OUT/prof$n
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --no-cpu-baseline $args > $log 2>&1
      rc=$?
      if [ $rc -eq 0 ]; then
        tr=$(find $d -name "*kernel_trace.csv" | head -1)
        python3 tools/kernel_table.py $tr > $d/kernel_table.txt 2>&1 && python3 tools/roofline_check.py $tr $log $OUT/roofline_check.json; rc=$?
      fi ;;
    pmc)
      d=$OUT/pmc$n
      a="--config ${cfg:-c3} --steps 3 --warmup 2 --no-cpu-baseline --no-sweep $args"
      rc=0
      for c in FETCH_SIZE WRITE_SIZE; do
        kt=""; [ $c = FETCH_SIZE ] && kt="--kernel-trace"
        timeout -s KILL 300 rocprofv3 $kt --pmc $c -d $d/$c -o run --output-format csv -- python3 bench.py $a > $d.$c.log 2>&1
        rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && break
      done
      if [ $rc -eq 0 ]; then
        timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE -d $d/MFMA -o run --output-format csv -- python3 bench.py $a > $d.MFMA.log 2>&1
        rc=$?; echo "MFMA rc=$rc"
      fi
      [ $rc -eq 0 ] && python3 tools/pmc_summary.py $d $OUT/pmc_traffic_${cfg:-c3}.json ${cfg:-c3} $d.FETCH_SIZE.log > $log 2>&1; rc=$? ;;
    sq|sqlds)
      # SQ instruction counts + kernel durations in one counter pass (serialised kernels) -> VALU roofline;
      # sqlds: LDS-array cycles / bank conflicts / waits instead
      d=$OUT/sq$n
      ctr="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
      [ $kind = sqlds ] && ctr="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
      timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $ctr \
        -d $d -o run --output-format csv -- python3 bench.py --config ${cfg:-c3} --steps 3 --warmup 2 --no-cpu-baseline --no-sweep $args > $log 2>&1
      rc=$?
      [ $rc -eq 0 ] && python3 tools/sq_summary.py $d $OUT/${kind}_${cfg:-c3}.json ${cfg:-c3} 2>&1 | tee -a $log; rc=${PIPESTATUS[0]} ;;
    ab)
      IFS=: read -r cfg pairs spec <<< "$rest"
      rc=0
      for i in $(seq 1 ${pairs:-4}); do
        for side in A B; do
          [ $side = A ] && sets=${spec%%/*} || sets=${spec#*/}
          sa=()
          if [ "$sets" != "-" ]; then IFS=, read -ra kv <<< "$sets"; for x in "${kv[@]}"; do sa+=(--set "$x"); done; fi
          timeout -k 10 600 python3 -u bench.py --config ${cfg:-c3} --no-cpu-baseline --no-sweep "${sa[@]}" > $OUT/ab$n.$side.$i.log 2>&1
          rc=$?; [ $rc -ne 0 ] && break 2
        done
      done
      [ $rc -eq 0 ] && python3 tools/bsum.py $OUT/ab$n.*.log | tee $log ;;
    abl)
      IFS=: read -r cfg pairs spec <<< "$rest"
      rc=0
      for i in $(seq 1 ${pairs:-4}); do
        for side in A B; do
          [ $side = A ] && b=${spec%%/*} || b=${spec#*/}
          [ "$b" = "-" ] && b=_build
          SNG_LIB_PATH=synerfgine_amd/$b/libsng_hip.so timeout -k 10 600 python3 -u bench.py --config ${cfg:-c3} --no-cpu-baseline --no-sweep > $OUT/abl$n.$side.$i.log 2>&1
          rc=$?; [ $rc -ne 0 ] && break 2
        done
      done
      [ $rc -eq 0 ] && python3 tools/bsum.py $OUT/abl$n.*.log | tee $log ;;
    sqpy)
      # the SQ pass over python3 tools/SCRIPT ARGS (e.g. train_bench.py) + tools/sq_summary.py
      d=$OUT/sq$n
      ctr="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
      timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $ctr -d $d -o run --output-format csv -- python3 tools/$cfg $args > $log 2>&1
      rc=$?
      [ $rc -eq 0 ] && python3 tools/sq_summary.py $d $OUT/sq_${cfg%.py}.json ${cfg%.py} 2>&1 | tee -a $log; rc=${PIPESTATUS[0]} ;;
    py)
      timeout -k 10 600 python3 -u tools/$cfg $args > $log 2>&1
      rc=$?; tail -c 3000 $log; echo ;;
    profpy)
      d=$OUT/prof$n
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 tools/$cfg $args > $log 2>&1
      rc=$?
      [ $rc -eq 0 ] && python3 tools/kernel_table.py $(find $d -name "*kernel_trace.csv" | head -1) > $d/kernel_table.txt 2>&1 && head -30 $d/kernel_table.txt ;;
    pmcpy)
      d=$OUT/pmc$n
      rc=0
      for c in FETCH_SIZE WRITE_SIZE; do
        kt=""; [ $c = FETCH_SIZE ] && kt="--kernel-trace"
        timeout -s KILL 300 rocprofv3 $kt --pmc $c -d $d/$c -o run --output-format csv -- python3 tools/$cfg $args > $d.$c.log 2>&1
        rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && break
      done
      if [ $rc -eq 0 ]; then
        timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE -d $d/MFMA -o run --output-format csv -- python3 tools/$cfg $args > $d.MFMA.log 2>&1
        rc=$?; echo "MFMA rc=$rc"
      fi
      [ $rc -eq 0 ] && python3 tools/pmc_summary.py $d $OUT/pmc_${cfg%.py}.json ${cfg%.py} > $log 2>&1; rc=$? ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  echo "[gpu.sh] step $n rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
