"""Per-iteration march log of one frame (param march_log): alive rays, steps and samples of every
trace_alt iteration, summarised by phase (head / one-step regime / multi-step / tail).

usage: python3 tools/march_log.py [c2|c3|c4] [KEY=VALUE ...]
"""
import json
import sys

sys.path.insert(0, "/root/repo")
import numpy as np

from synerfgine_amd import scene as S

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
ov = {"march_log": 1, "concurrent_streams": 0}
for kv in sys.argv[2:]:
    k, v = kv.split("=")
    ov[k] = float(v)
tb, eng, _ = S.make_engine(cfg, overrides=ov)
for _ in range(3):
    r = eng.frame(collect_kernel_times=True)
log = eng.frame_buffer("march_log", np.uint32).reshape(-1, 3)
n = r.n_iterations
log = log[:n]
print(json.dumps({"config": cfg, "ms_frame": r.ms_frame, "nerf_ms": r.ms_nerf, "iterations": n, "network_launches": r.network_launches}))
i_step = 1
rows = []
for k, (alive, steps, samples) in enumerate(log):
    rows.append((k, int(alive), int(steps), int(samples), i_step))
    i_step += int(steps)
# print a compressed view: every iteration whose steps differ from the previous, plus every 50th
prev = None
for k, alive, steps, samples, i in rows:
    if steps != prev or k % 50 == 0 or k == n - 1:
        print(f"iter {k:5d}  i {i:5d}  alive {alive:8d}  steps {steps}  samples {samples:9d}")
    prev = steps
multi = [x for x in rows if x[2] > 1]
print("multi-step iterations:", len(multi), "steps", sum(x[2] for x in multi), "samples", sum(x[3] for x in multi),
      "alive range", (multi[0][1], multi[-1][1]) if multi else None)
tb.close()
