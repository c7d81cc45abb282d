set -o pipefail
bash tools/closing.sh 1 || exit 1
for v in nonerf nobvh; do
  SNG_LIB_PATH=synerfgine_amd/_build_$v/libsng_hip.so TAG=r04m_$v tools/gpu.sh prof:c3:--serial-streams > /dev/null 2>&1 || exit 1
  echo "== $v"; grep -E "raytrace_kernel|shadow_rays" gpurun_out/r04m_$v/prof1/kernel_table.txt
done
