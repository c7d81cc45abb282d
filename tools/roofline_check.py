"""Recompute the driver line's roofline fields from a rocprofv3 kernel trace of the SAME bench.py process.

bench.py times the network launches with dispatch-recorded HIP events; this reads the kernel trace rocprofv3 wrote
for the same run (tools/gpu.sh profdriver) and forms, from its own durations, the fraction each field quotes:
  timed region   nerf_network_kernel launches of the warm-up + timed frames, the timed ones only (the line's launch counts)
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
# the warm-up frames' launches as the line counted them (their number per frame can differ from the timed frames':
# the first frame has no last-frame statistics for nerf_spec_adapt); older lines: the timed frames' rate
n0 = int(rf["warmup_launches"]) if "warmup_launches" in rf else int(round(per_frame * w))
n1 = n0 + int(rf["launches"])
timed = dur[n0:n1]
bytes_per_launch = rf["samples_in_launches"] / rf["launches"] * rf["algorithmic_bytes_per_sample"]
res = {"bench_line_value": line["value"], "samples_per_launch": rf["samples_in_launches"] / rf["launches"],
       "algorithmic_bytes_per_launch": bytes_per_launch,
       "timed": {"launches": len(timed), "rocprof_avg_ms": sum(timed) / len(timed) * 1e3, "hipevent_avg_ms": rf["avg_launch_ms"]}}
res["timed"]["rocprof_frac"] = bytes_per_launch / (res["timed"]["rocprof_avg_ms"] * 1e-3) / (rf["peak"] * 1e9)
res["timed"]["line_frac"] = rf["frac"]
BPS = rf["algorithmic_bytes_per_sample"]
ppf = int(round(per_frame))


def per_launch(durs, line_rows, n_per_frame=None):
    """durations grouped by launch index within the frame (a fixed number of launches per frame), against the
    line's own per-launch rows (HIP events; samples read by the kernel)"""
    n = ppf if n_per_frame is None else n_per_frame
    if n < 1 or (n_per_frame is None and abs(per_frame - ppf) > 1e-6) or not line_rows:
        return None
    out = []
    for k in range(n):
        d = durs[k::n]
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
    # the serialized leg's own launches per frame (its per-launch rows): a serialized frame may keep a speculative round
    # the concurrent frames drop (nerf_spec_adapt acts on hybrid concurrent frames only)
    alt = (unc.get("alternates") or {}).get("hip_events_this_process") or {}
    rows_u = alt.get("per_launch") or []
    ppf_u = len(rows_u) if rows_u else ppf
    l0 = n1 + int(unc.get("warmup_launches", ppf_u * 2))   # frame_cells: 2 warm-up + 10 frames
    leg = dur[l0:l0 + int(unc.get("launches", ppf_u * 10))]
    if leg:
        pl = per_launch(leg, rows_u, ppf_u)
        if pl:   # sample-weighted over the frame's launches, as the line's figure
            byts = sum(r["samples"] * BPS for r in pl)
            secs = sum(r["rocprof_ms"] for r in pl) * 1e-3
            a = secs / len(pl)
            frac = byts / secs / (rf["peak"] * 1e9)
        else:
            a = sum(leg) / len(leg)
            frac = bytes_per_launch / a / (rf["peak"] * 1e9)
        res["uncontended"] = {"launches": len(leg), "launches_per_frame": ppf_u, "rocprof_avg_ms": a * 1e3, "rocprof_frac": frac,
                              "line_frac": alt.get("frac", unc["frac"]), "per_launch": pl}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
