"""tools/roofline_check.py aligns a rocprofv3 kernel trace with the bench line of the same process: the warm-up frames'
network launches (whose count per frame can differ from the timed frames': the first frame has no last-frame
statistics for nerf_spec_adapt), the timed launches, then the serialized leg with its own launches per frame.  A
synthetic trace with known durations checks that each figure is formed from the launches it names."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BPS = 548
PEAK = 8000.0


def _write(tmp, warm, timed, leg_warm, leg, after):
    """each list holds (samples, duration_ns) per network launch, in dispatch order"""
    rows, t = [], 1000
    for s, d in warm + timed + leg_warm + leg + after:
        rows.append({"Kernel_Name": "sng::nerf_network_kernel<4, 1, false>", "Start_Timestamp": t, "End_Timestamp": t + d})
        rows.append({"Kernel_Name": "sng::raytrace_kernel", "Start_Timestamp": t + 1, "End_Timestamp": t + 5})
        t += d + 100
    tr = os.path.join(tmp, "trace.csv")
    with open(tr, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)
    n_t = len(timed)
    samples = sum(s for s, _ in timed)
    line = {"metric": "m", "value": 1.0, "steps": n_t, "warmup": 3,
            "roofline": {"frac": 0.5, "peak": PEAK, "launches": n_t, "warmup_launches": len(warm), "samples_in_launches": samples,
                         "algorithmic_bytes_per_sample": BPS, "avg_launch_ms": 0.16,
                         "per_launch": [{"index": 0, "frames": n_t, "samples": timed[0][0], "ms": 0.16, "frac": 0.5}],
                         "uncontended": {"frac": 0.6, "warmup_launches": len(leg_warm), "launches": len(leg),
                                         "alternates": {"hip_events_this_process": {"frac": 0.59, "per_launch": [
                                             {"index": 0, "frames": 10, "samples": leg[0][0], "ms": 0.13, "frac": 0.6},
                                             {"index": 1, "frames": 10, "samples": leg[1][0], "ms": 0.011, "frac": 0.0007}]}}}}}
    log = os.path.join(tmp, "bench.log")
    with open(log, "w") as f:
        f.write("some output\n" + json.dumps(line) + "\n")
    return tr, log


def test_alignment_with_uneven_warmup_and_serial_leg(tmp_path):
    big, small = 1200502, 111
    warm = [(big, 200000), (small, 15000), (big, 190000), (big, 180000)]        # 3 frames, the first with two rounds
    timed = [(big, 150000)] * 20                                                # one launch per concurrent frame
    leg_warm = [(big, 130000), (small, 7000)] * 2                               # serialized: both rounds kept
    leg = [(big, 125000), (small, 6000)] * 10
    after = [(big, 999999)] * 5                                                 # later legs of the same process
    tr, log = _write(str(tmp_path), warm, timed, leg_warm, leg, after)
    out = os.path.join(str(tmp_path), "rc.json")
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "roofline_check.py"), tr, log, out], check=True, capture_output=True)
    r = json.load(open(out))
    assert r["timed"]["launches"] == 20
    assert abs(r["timed"]["rocprof_avg_ms"] - 0.150) < 1e-9
    assert abs(r["timed"]["rocprof_frac"] - big * BPS / 150e-6 / (PEAK * 1e9)) < 1e-9
    u = r["uncontended"]
    assert u["launches"] == 20 and u["launches_per_frame"] == 2
    pl = u["per_launch"]
    assert [p["samples"] for p in pl] == [big, small]
    assert abs(pl[0]["rocprof_ms"] - 0.125) < 1e-9 and abs(pl[1]["rocprof_ms"] - 0.006) < 1e-9
    assert abs(u["rocprof_frac"] - (big + small) * BPS / 131e-6 / (PEAK * 1e9)) < 1e-9
