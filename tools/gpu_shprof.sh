#!/bin/bash
# shadow-kernel cost attribution: kernel tables under several overrides
for cfg in "" "n_steps=0" "n_steps=1" "syn_shadow_samples=1"; do
  echo "### $cfg"
  bash tools/gpu_rtprof.sh "$cfg" | grep -E "rc=|shadow_rays|raytrace_kernel|rt_accum" || exit 1
  rm -rf gpurun_out/rtprof
done
