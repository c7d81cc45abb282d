#!/bin/bash
# Issue/stall breakdown of the traversal kernels (C3, serialized streams): one SQ pass, kernel trace only.
# usage: tools/gpu_pmc_rt.sh [tag] [config]
tag=${1:-pmc_rt}
export TMPDIR=/tmp
d=gpurun_out/$tag
mkdir -p $d
args="--config ${2:-c3} --steps 3 --warmup 1 --no-cpu-baseline --no-sweep --serial-streams"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS \
  -d $d/sq -o run --output-format csv -- python3 bench.py $args > $d/sq.log 2>&1 || { tail -20 $d/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
  -d $d/sq2 -o run --output-format csv -- python3 bench.py $args > $d/sq2.log 2>&1 || { tail -20 $d/sq2.log; exit 1; }
python3 - $d <<'EOF'
import csv, glob, sys
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
n = defaultdict(int)
for f in glob.glob(d + "/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not any(s in k for s in ("shadow_rays_kernel", "raytrace_kernel", "nerf_fused_kernel", "rt_accumulate", "shade_shadow", "onestep_kernel", "generate_kernel")):
            continue
        acc[k[:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    print(k)
    print("   ", {a: f"{b:.4g}" for a, b in sorted(c.items())})
    w = c.get("SQ_WAVE_CYCLES", 0)
    if w:
        print("    frac of wave cycles: wait_any %.3f wait_inst_any %.3f active_any %.3f active_valu %.3f wait_inst_lds %.3f active_lds %.3f" % tuple(
            c.get(x, 0) / w for x in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS")))
EOF
