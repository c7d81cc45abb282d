"""Device time per training step from a rocprofv3 kernel trace of tools/train_trace.py (20 warmup steps, 60 timed
steps, then 50 steps with per-stage timing): python tools/train_gaps.py <kernel_trace.csv>. Over the 60 timed steps
(from the 20th train_adam_kernel to the 80th): span, busy and idle time per step, the largest idle gaps with the
kernels on either side, and each kernel's time per step (the density-grid update's kernels run every few steps)."""
import csv
import sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ad = [i for i, r in enumerate(rows) if "train_adam_kernel" in r["Kernel_Name"]]
a0, a1 = ad[19], ad[79]
seg = rows[a0 + 1:a1 + 1]
n = 60
t0, t1 = int(rows[a0]["End_Timestamp"]), int(seg[-1]["End_Timestamp"])
busy, end, gaps, prev = 0, t0, {}, rows[a0]
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s > end:
        k = (prev["Kernel_Name"][:50], r["Kernel_Name"][:50])
        gaps[k] = gaps.get(k, 0) + s - end
    busy += max(0, e - max(s, end))
    end = max(end, e)
    prev = r
print(f"timed steps {n}: span {(t1 - t0) / n / 1e3:.1f} us/step, busy {busy / n / 1e3:.1f}, idle {(t1 - t0 - busy) / n / 1e3:.1f}")
print("largest gaps (us/step):")
for (a, b), g in sorted(gaps.items(), key=lambda x: -x[1])[:6]:
    print(f"  {g / n / 1e3:7.2f}  {a}  ->  {b}")
tot, cnt = {}, {}
for r in seg:
    k = r["Kernel_Name"][:60]
    tot[k] = tot.get(k, 0) + int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    cnt[k] = cnt.get(k, 0) + 1
print("kernels (us/step, launches, us/launch):")
for k, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {v / n / 1e3:8.2f}  {cnt[k]:4d}  {v / cnt[k] / 1e3:7.1f}  {k}")
