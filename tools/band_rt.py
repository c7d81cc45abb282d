"""Raytracer stage time of one thin band under overrides (serialized streams)."""
import json
import sys

sys.path.insert(0, "/root/repo")
from synerfgine_amd import scene as S

r0, r1 = int(sys.argv[1]), int(sys.argv[2])
CASES = [{}, {"light_samples": 1}] if len(sys.argv) > 3 else [{}, {"light_samples": 1}, {"light_samples": 2}, {"light_samples": 4}, {"path_trace_depth": 1}, {"syn_shadow_samples": 1},
         {"rt_tile_order": 0}, {"scene_lds": 0}, {"rt_wavefront": 0}]
tb, eng, _ = S.make_engine("c3", overrides={"concurrent_streams": 0})
base = {k: eng.get_param(k) for c in CASES for k in c}
for ov in CASES:
    for k, v in {**base, **ov}.items():
        eng.set_param(k, v)
    ts = []
    for _ in range(5):
        r = eng.frame(rows=(r0, r1))
        ts.append(r.ms_raytrace)
    print(json.dumps({"rows": [r0, r1], "overrides": ov, "ms_raytrace": round(min(ts[1:]), 3)}), flush=True)
tb.close()
