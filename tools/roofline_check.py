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
BPS = rf["algorithmic_bytes_per_sample"]
ppf = int(round(per_frame))


def per_launch(durs, line_rows):
    """durations grouped by launch index within the frame (a fixed number of launches per frame), against the
    line's own per-launch rows (HIP events; samples read by the kernel)"""
    if ppf < 1 or abs(per_frame - ppf) > 1e-6 or not line_rows:
        return None
    out = []
    for k in range(ppf):
        d = durs[k::ppf]
        lr = next((r for r in line_rows if r["index"] == k), None)
        if not d or not lr:
            continue
        ms = sum(d) / len(d) * 1e3
        out.append({"index": k, "launches": len(d), "samples": lr["samples"], "rocprof_ms": ms, "hipevent_ms": lr["ms"],
                    "rocprof_frac": lr["samples"] * BPS / (ms * 1e-3) / (rf["peak"] * 1e9), "hipevent_frac": lr["frac"],
                    "hipevent_over_rocprof": lr["ms"] / ms})
    return out


res["timed"]["per_launch"] = per_launch(timed, rf.get("per_launch"))
unc = rf.get("uncontended")
if unc and "frac" in unc:
    leg = dur[n1 + int(round(per_frame * 2)):n1 + int(round(per_frame * 12))]   # 2 warm-up + 10 frames of frame_cells
    if leg:
        a = sum(leg) / len(leg)
        alt = (unc.get("alternates") or {}).get("hip_events_this_process") or {}
        res["uncontended"] = {"launches": len(leg), "rocprof_avg_ms": a * 1e3, "rocprof_frac": bytes_per_launch / a / (rf["peak"] * 1e9),
                              "line_frac": alt.get("frac", unc["frac"]), "per_launch": per_launch(leg, alt.get("per_launch"))}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
