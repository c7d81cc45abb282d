"""One band of an N-way split rendered repeatedly under the replayed frame-wide schedule (as tools/band8.py times it),
for rocprofv3 kernel tables of a rank's frame: python tools/band_prof.py --config c4 --bounds 769-844 [--frames 10]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from synerfgine_amd import scene as S  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c4")
ap.add_argument("--bounds", default="769,844")
ap.add_argument("--frames", type=int, default=10)
ap.add_argument("--set", action="append", default=[])
args = ap.parse_args()
model = "lego" if args.config != "c4" else "synthetic"
ov = {kv.split("=")[0]: float(kv.split("=")[1]) for kv in args.set}
tb, eng, _ = S.make_engine(args.config, model=model, overrides=ov)
rows = tuple(int(x) for x in args.bounds.replace("-", ",").split(","))
log = eng.record_schedule()
recs = []
for _ in range(2):
    eng.frame()
    recs.append(list(log))
    log.clear()
eng.detach_comm()
eng.set_sched_replay(recs[0])
eng.frame(rows=rows)
eng.set_sched_replay(recs[1])
eng.frame(rows=rows)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(args.frames):
    r = eng.frame(rows=rows, collect_kernel_times=True)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / args.frames * 1e3
print(json.dumps({"config": args.config, "rows": rows, "ms": round(ms, 3), "device_ms": round(r.ms_frame, 3), "nerf_ms": round(r.ms_nerf, 3),
                  "shadow_ms": round(r.ms_shadow, 3), "raytrace_ms": round(r.ms_raytrace, 3), "iterations": r.n_iterations,
                  "onestep": [r.onestep_from_iter, r.onestep_iterations], "ms_onestep": round(r.ms_onestep, 3), "msr_rounds": r.msr_rounds,
                  "network_launches": r.network_launches, "ms_network": round(r.ms_network, 3), "reductions": r.sched_reductions}), flush=True)
eng.set_sched_replay(None)
tb.close()
