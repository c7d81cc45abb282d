"""Tail diagnostics: per-iteration alive / sample histograms and the speculative rounds' statistics for a config,
and the frame time for a list of parameter sets.

usage: python tools/tail_diag.py CONFIG [key=value+key=value ...]   (one parameter set per argument; none: defaults)
"""
import json
import sys
import time

sys.path.insert(0, "/root/repo")
import torch

from synerfgine_amd import scene as S

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
sets = [dict((kv.split("=")[0], float(kv.split("=")[1])) for kv in a.split("+") if kv) for a in sys.argv[2:]] or [{}]
tb, eng, _ = S.make_engine(cfg, model="lego" if cfg != "c4" else "synthetic")
first = True
for ov in sets:
    for k, v in ov.items():
        eng.set_param(k, v)
    for _ in range(3):
        r = eng.frame(collect_kernel_times=True)
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        r = eng.frame(collect_kernel_times=True)
    torch.cuda.synchronize()
    fps = n / (time.perf_counter() - t0)
    if first:
        print("alive  ", r.alive_per_iter)
        print("samples", r.samples_per_iter)
        first = False
    print(json.dumps({"set": ov, "fps": round(fps, 1), "ms_frame": round(r.ms_frame, 3), "nerf": round(r.ms_nerf, 3),
                      "raytrace": round(r.ms_raytrace, 3), "net_ms": round(r.ms_network, 4), "launches": r.network_launches,
                      "tail_ms": round(r.ms_fused_tail, 4), "spec_evals": r.spec_evals, "spec_exec": r.spec_exec,
                      "iters": r.n_iterations, "samples": r.n_samples}), flush=True)
if any(ov.get("nerf_spec_debug") for ov in sets):
    import numpy as np
    W, H = eng.resolution()["nerf"]
    dbg = eng.frame_buffer("spec_dbg", np.uint32).reshape(-1, W * H, 4)   # [round][pixel] {trips, samples|loads<<16, cycles, A bits}
    alive = dbg[:, :, 0] > 0
    for r, d in enumerate(dbg):
        m = alive[r]
        if not m.any():
            continue
        d = d[m]
        cyc = d[:, 2].astype(np.float64)
        tr = d[:, 0].astype(np.float64)
        am = int(np.argmax(tr))
        print(json.dumps({"round": r, "rays": int(m.sum()), "trips_max": int(tr.max()), "trips_mean": round(tr.mean(), 1),
                          "trips_p99": float(np.percentile(tr, 99)), "samples_max": int((d[:, 1] & 0xffff).max()), "cycles_max": int(cyc.max()),
                          "cycles_per_trip_of_max": round(float(cyc[am] / tr.max()), 1)}))
    # rounds of one iteration each (nerf_spec_kmax=1): remaining iterations of the rays alive after the head vs their opacity
    if alive.shape[0] > 1:
        a0 = dbg[0, :, 3].view(np.float32)
        rem = alive.sum(axis=0)
        m = alive[0]
        for lo, hi in ((0, 0.05), (0.05, 0.2), (0.2, 0.5), (0.5, 0.8), (0.8, 0.95), (0.95, 1.01)):
            sel = m & (a0 >= lo) & (a0 < hi)
            if sel.any():
                q = rem[sel]
                print(json.dumps({"A_after_head": [lo, hi], "rays": int(sel.sum()), "iters_mean": round(float(q.mean()), 2),
                                  "iters_p50": float(np.percentile(q, 50)), "iters_p90": float(np.percentile(q, 90)), "iters_max": int(q.max()),
                                  "frac_1": round(float((q == 1).mean()), 3)}))
tb.close()
