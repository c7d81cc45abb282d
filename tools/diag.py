"""GPU diagnostics: stage times (streams serialized), wavefront statistics, standalone network throughput."""
import json
import sys
import time

sys.path.insert(0, "/root/repo")
import numpy as np
import torch

from synerfgine_amd import scene as S

tb, eng, _ = S.make_engine("c3", overrides={"concurrent_streams": 0})
for i in range(3):
    r = eng.frame(collect_kernel_times=True)
print(json.dumps({"ms_frame": r.ms_frame, "raytrace": r.ms_raytrace, "nerf": r.ms_nerf, "shadow": r.ms_shadow, "overlay": r.ms_overlay,
                  "network_sum": r.ms_network, "launches": r.network_launches, "iters": r.n_iterations, "samples": r.n_samples,
                  "hit": r.n_hit}))
print("alive", r.alive_per_iter)
print("steps", r.steps_per_iter)
print("samples", r.samples_per_iter)
# standalone network on random coordinates
for n in (1 << 20, 1 << 22):
    rng = np.random.default_rng(0)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = rng.uniform(0.2, 0.8, (n, 3))
    c[:, 3] = 0.0
    c[:, 4:] = rng.uniform(0, 1, (n, 3))
    dc = torch.from_numpy(c).cuda()
    out = torch.empty((n, 4), dtype=torch.float16, device="cuda")
    for _ in range(3):
        tb.inference_mixed_precision(dc.data_ptr(), 7, n, out.data_ptr(), layout=1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        tb.inference_mixed_precision(dc.data_ptr(), 7, n, out.data_ptr(), layout=1)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    print(f"network standalone n={n}: {dt*1e3:.3f} ms  {n/dt/1e9:.3f} Gsamples/s  {n*548/dt/1e9:.1f} GB/s algorithmic  {n*20480/dt/1e12:.1f} TFLOP/s")
tb.close()
