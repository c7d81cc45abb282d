#!/bin/bash
# per-wave SQ counters of the kernels of one thin band frame loop: tools/gpu_sqband.sh R0 R1
export TMPDIR=/tmp
mkdir -p gpurun_out/sqb
r0=${1:-560}; r1=${2:-568}
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES" \
           "SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc -d gpurun_out/sqb/p$i -o run --output-format csv -- python3 tools/small_band.py $r0 $r1 serial > gpurun_out/sqb/log$i 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/sqb/log$i; exit $rc; }
done
python3 - <<'PY'
import csv, glob, re
from collections import defaultdict
agg = defaultdict(lambda: defaultdict(float))
for f in glob.glob("gpurun_out/sqb/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("sng::", "")[:34]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        agg[k]["_n_" + r["Counter_Name"]] += 0
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:8]:
    w = max(v.get("SQ_WAVES", 1), 1)
    print(k, "waves", int(w), " ".join(f"{c.replace('SQ_', '')}={v[c] / w:.0f}" for c in sorted(v) if c.startswith("SQ_") and c != "SQ_WAVES"))
PY
