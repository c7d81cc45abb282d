"""Device-idle time per training step from a rocprofv3 kernel trace (tools/train_trace.py):
python tools/train_gaps.py <kernel_trace.csv>. Prints the busy / idle split between consecutive dispatches of the
last 60 steps (from the 60th-last train_adam_kernel on) and the largest gaps with the kernels on either side."""
import csv
import sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ad = [i for i, r in enumerate(rows) if "train_adam_kernel" in r["Kernel_Name"]]
i0 = ad[-61] + 1
seg = rows[i0:ad[-1] + 1]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
busy, gaps, end = 0, [], t0
for a, b in zip([rows[i0 - 1]] + seg[:-1], seg):
    s, e = int(b["Start_Timestamp"]), int(b["End_Timestamp"])
    if s > end:
        gaps.append((s - end, a["Kernel_Name"][:60], b["Kernel_Name"][:60]))
    busy += max(0, e - max(s, end))
    end = max(end, e)
n = 60
print(f"steps {n}: span {(t1 - t0) / n / 1e3:.1f} us/step, busy {busy / n / 1e3:.1f}, idle {(t1 - t0 - busy) / n / 1e3:.1f}")
agg = {}
for g, a, b in gaps:
    k = (a, b)
    agg[k] = agg.get(k, 0) + g
for (a, b), g in sorted(agg.items(), key=lambda x: -x[1])[:15]:
    print(f"{g / n / 1e3:8.2f} us/step  {a}  ->  {b}")
