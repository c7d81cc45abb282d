"""Render one band (or the full frame) of the C3 lego frame repeatedly under engine overrides, for
rocprofv3 kernel statistics.  python tools/band_kernels.py r0 r1 [k=v,k=v] [frames]"""
import json
import sys
import time

sys.path.insert(0, "/root/repo")
import torch

from synerfgine_amd import scene as S

r0, r1 = int(sys.argv[1]), int(sys.argv[2])
ov = dict((kv.split("=")[0], float(kv.split("=")[1])) for kv in sys.argv[3].split(",") if kv) if len(sys.argv) > 3 else {}
n = int(sys.argv[4]) if len(sys.argv) > 4 else 20
tb, eng, _ = S.make_engine("c3", overrides=ov, model="lego")
H = eng.resolution()["mesh"][1]
rows = None if (r0, r1) == (0, H) else (r0, r1)
for _ in range(3):
    eng.frame(rows=rows)
torch.cuda.synchronize()
t0 = time.perf_counter()
rs = [eng.frame(rows=rows) for _ in range(n)]
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / n * 1e3
print(json.dumps({"rows": [r0, r1], "overrides": ov, "ms_frame": round(ms, 3), "ms_raytrace": round(sum(r.ms_raytrace for r in rs) / n, 3),
                  "ms_nerf": round(sum(r.ms_nerf for r in rs) / n, 3)}), flush=True)
tb.close()
