#!/bin/bash
# tools/closing.sh -- the round's closing measurements on one GPU box, in three parts (one gpurun call each), so that
# every roofline field of the driver line recomputes from profiles/ of the build that is timed.
#   part 1: C3 -- concurrent + serialized rocprofv3 kernel tables, PMC traffic (FETCH/WRITE/MFMA) with the counted
#           run's own samples per launch, SQ instruction and LDS passes
#   part 2: C4 -- kernel tables, SQ + PMC passes; nerf_views legs and C5 training under rocprofv3 (+ training PMC)
#   part 3: the band split under the replayed frame-wide schedule, C3 and C4 at N = 2 / 4 / 8
# usage (inside gpurun): tools/closing.sh 1|2|3      output: gpurun_out/r04c{1,2,3}/
set -o pipefail
part=${1:-1}
case $part in
  1) TAG=r04c1 tools/gpu.sh prof:c3 prof:c3:--serial-streams pmc:c3 sq:c3 sqlds:c3 ;;
  2) TAG=r04c2 tools/gpu.sh bench:c4 prof:c4 sq:c4 pmc:c4 profpy:views_bench.py:10 profpy:train_bench.py:200,50 pmcpy:train_bench.py:30,20 ;;
  3) TAG=r04c3 tools/gpu.sh py:band8.py:--n,2,--config,c4,--out,gpurun_out/r04c3/band_split.jsonl \
       py:band8.py:--n,4,--config,c4,--out,gpurun_out/r04c3/band_split.jsonl \
       py:band8.py:--n,8,--config,c4,--out,gpurun_out/r04c3/band_split.jsonl \
       py:band8.py:--n,2,--config,c3,--out,gpurun_out/r04c3/band_split.jsonl \
       py:band8.py:--n,4,--config,c3,--out,gpurun_out/r04c3/band_split.jsonl \
       py:band8.py:--n,8,--config,c3,--cases,/rt_tile=4,--out,gpurun_out/r04c3/band_split.jsonl ;;
  *) echo "part 1, 2 or 3"; exit 2 ;;
esac
