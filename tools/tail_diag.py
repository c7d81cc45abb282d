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
tb.close()
