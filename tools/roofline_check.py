"""Recompute the driver line's roofline fields from a rocprofv3 kernel trace of the SAME bench.py process.

bench.py times the network launches with dispatch-recorded HIP events; this reads the kernel trace rocprofv3 wrote
for the same run (tools/gpu.sh profdriver) and forms, from its own durations, the fraction each field quotes:
  timed region   nerf_network_kernel launches of the warm-up + timed frames (2 per C3 frame), the timed ones only
  uncontended    the launches of the serialized leg that follows the timed region (2 warm-up + 10 frames)
usage: python tools/roofline_check.py <kernel_trace.csv> <bench log with the JSON line> <out.json>"""
import csv
import json
import sys

trace, log, out = sys.argv[1:4]
line = None
for l in open(log):
    if l.startswith('{"metric"'):
        line = json.loads(l)
rf = line["roofline"]
per_frame = rf["launches"] / line["steps"]
rows = [r for r in csv.DictReader(open(trace)) if "nerf_network_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in rows]
w, k = line["warmup"], line["steps"]
n0 = int(round(per_frame * w))
n1 = int(round(per_frame * (w + k)))
timed = dur[n0:n1]
bytes_per_launch = rf["samples_in_launches"] / rf["launches"] * rf["algorithmic_bytes_per_sample"]
res = {"bench_line_value": line["value"], "samples_per_launch": rf["samples_in_launches"] / rf["launches"],
       "algorithmic_bytes_per_launch": bytes_per_launch,
       "timed": {"launches": len(timed), "rocprof_avg_ms": sum(timed) / len(timed) * 1e3, "hipevent_avg_ms": rf["avg_launch_ms"]}}
res["timed"]["rocprof_frac"] = bytes_per_launch / (res["timed"]["rocprof_avg_ms"] * 1e-3) / (rf["peak"] * 1e9)
res["timed"]["line_frac"] = rf["frac"]
unc = rf.get("uncontended")
if unc and "frac" in unc:
    leg = dur[n1 + int(round(per_frame * 2)):n1 + int(round(per_frame * 12))]   # 2 warm-up + 10 frames of frame_cells
    if leg:
        a = sum(leg) / len(leg)
        res["uncontended"] = {"launches": len(leg), "rocprof_avg_ms": a * 1e3, "rocprof_frac": bytes_per_launch / a / (rf["peak"] * 1e9),
                              "line_frac": unc["frac"]}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
