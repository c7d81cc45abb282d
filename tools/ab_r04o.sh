set -o pipefail
TAG=r04bp tools/gpu.sh profpy:band_prof.py:--config,c4,--bounds,766-841 py:tile_cost.py:--config,c3,--bounds,498-558 > /dev/null 2>&1; rc=$?
grep '^{' gpurun_out/r04bp/1.profpy.log | tail -1; head -16 gpurun_out/r04bp/prof1/kernel_table.txt; grep '^{' gpurun_out/r04bp/2.py.log; exit $rc
