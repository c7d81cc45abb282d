"""Raytracer stage time of bands under rt_spec 0/1 (serialized streams, lego C3).
python tools/spec_probe.py [r0:r1 ...]"""
import json
import sys
import time

sys.path.insert(0, "/root/repo")
import torch

from synerfgine_amd import scene as S

tb, eng, _ = S.make_engine("c3", overrides={"concurrent_streams": 0}, model="lego")
H = eng.resolution()["mesh"][1]
bands = [tuple(int(v) for v in b.split(":")) for b in sys.argv[1:]] or [(500, 508), (491, 551), (348, 430), (0, H)]
for r0, r1 in bands:
    rows = None if (r0, r1) == (0, H) else (r0, r1)
    res = {}
    for spec in (0, 1):
        eng.set_param("rt_spec", spec)
        for _ in range(3):
            eng.frame(rows=rows)
        torch.cuda.synchronize()
        rs = [eng.frame(rows=rows) for _ in range(10)]
        res[spec] = round(sum(r.ms_raytrace for r in rs) / len(rs), 3)
    print(json.dumps({"rows": [r0, r1], "rt_ms_serial": res[0], "rt_ms_spec": res[1]}), flush=True)
tb.close()
