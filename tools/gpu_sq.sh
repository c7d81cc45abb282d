#!/bin/bash
# SQ counters (issue vs wait) for the hot kernels, one PMC pass, no traces
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d gpurun_out/sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --serial-streams > gpurun_out/sq/log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/sq/log; exit $rc; }
python3 - <<'PY'
import csv, glob, re
from collections import defaultdict
f = glob.glob("gpurun_out/sq/**/*counter_collection.csv", recursive=True)[0]
agg = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("sng::", "")[:40]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
cols = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"]
print("kernel".ljust(40), " ".join(c.replace("SQ_", "")[:12].rjust(13) for c in cols))
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"])[:10]:
    print(k.ljust(40), " ".join(f"{v[c]:13.3g}" for c in cols))
PY
