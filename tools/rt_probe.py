"""Raytracer latency probe: stage times of one band (or the full frame) under engine overrides
(serialized streams).  python tools/rt_probe.py r0 r1 ["k=v,k=v;k=v"]"""
import json
import sys
import time

sys.path.insert(0, "/root/repo")
import torch

from synerfgine_amd import scene as S

r0, r1 = int(sys.argv[1]), int(sys.argv[2])
cases = [""] + (sys.argv[3].split(";") if len(sys.argv) > 3 else [])
tb, eng, _ = S.make_engine("c3", overrides={"concurrent_streams": 0}, model="lego")
H = eng.resolution()["mesh"][1]
rows = None if (r0, r1) == (0, H) else (r0, r1)
base = {}
for c in cases:
    ov = dict((kv.split("=")[0], float(kv.split("=")[1])) for kv in c.split(",") if kv)
    for k, v in base.items():
        eng.set_param(k, v)
    for k in ov:
        base.setdefault(k, eng.get_param(k))
    for k, v in ov.items():
        eng.set_param(k, v)
    for _ in range(2):
        eng.frame(rows=rows)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rs = [eng.frame(rows=rows) for _ in range(5)]
    torch.cuda.synchronize()
    r = rs[-1]
    print(json.dumps({"ov": ov, "wall_ms": round((time.perf_counter() - t0) / 5 * 1e3, 3), "rt_ms": round(min(x.ms_raytrace for x in rs), 3),
                      "nerf_ms": round(min(x.ms_nerf for x in rs), 3)}), flush=True)
tb.close()
