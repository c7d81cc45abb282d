"""Render one thin band repeatedly (fixed per-frame cost analysis); optional serialized streams."""
import sys
import time

sys.path.insert(0, "/root/repo")
import torch

from synerfgine_amd import scene as S

r0, r1 = int(sys.argv[1]), int(sys.argv[2])
serial = len(sys.argv) > 3 and sys.argv[3] == "serial"
tb, eng, _ = S.make_engine("c3", overrides={"concurrent_streams": 0} if serial else None, model="lego")
for _ in range(3):
    eng.frame(rows=(r0, r1))
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    r = eng.frame(rows=(r0, r1), collect_kernel_times=True)
torch.cuda.synchronize()
print("band", (r0, r1), "ms/frame", (time.perf_counter() - t0) / 10 * 1e3, "dev ms", r.ms_frame, "rt", r.ms_raytrace, "nerf", r.ms_nerf,
      "iters", r.n_iterations, "alive", r.alive_per_iter[:6])
tb.close()
