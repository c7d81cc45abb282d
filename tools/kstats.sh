#!/bin/bash
# Per-kernel VGPR/SGPR/LDS/scratch usage of a HIP source (device-only compile for gfx950).
# usage: tools/kstats.sh synerfgine_amd/csrc/nerf.hip [filter]
set -e
src=$1; out=/tmp/kstats_$(basename "$src").co
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math $KEXTRA --cuda-device-only --no-gpu-bundle-output -c "$src" -o "$out"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$out" | grep -E "^\s+\.name:|\.vgpr_count|\.sgpr_count|\.private_segment_fixed_size|\.group_segment_fixed_size|\.vgpr_spill" | grep -A5 -E "${2:-.}" || true
