#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/band
timeout -k 10 200 python tools/small_band.py 907 1080 serial 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python tools/small_band.py 907 1080 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/band -o run --output-format csv -- python3 tools/small_band.py 907 1080 serial > gpurun_out/band/log 2>&1; echo "prof rc=$?"
python3 - <<'PY'
import csv, glob, re
f = glob.glob("gpurun_out/band/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# last frame: from the last ctrl_init to the end
idx = [i for i, r in enumerate(rows) if "ctrl_init" in r["Kernel_Name"]]
last = rows[idx[-2]:idx[-1]] if len(idx) > 1 else rows
t0 = int(last[0]["Start_Timestamp"])
busy = 0
prev_end = t0
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("sng::", "")[:34]
    gap = (s - prev_end) / 1e3
    print(f"{(s - t0) / 1e3:9.1f} us  gap {gap:7.1f}  dur {(e - s) / 1e3:8.1f}  {name}")
    busy += e - s
    prev_end = max(prev_end, e)
print("span us", (prev_end - t0) / 1e3, "busy us", busy / 1e3)
PY
