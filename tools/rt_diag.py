"""Raytracer cost attribution: ms_raytrace of config c3 under parameter overrides (streams serialized)."""
import json
import sys

sys.path.insert(0, "/root/repo")
import numpy as np

from synerfgine_amd import scene as S

CASES = [{}, {"rt_tile_order": 0}, {"rt_wavefront": 0}, {"scene_lds": 0}, {"shadow_on_virtual_obj": 0}, {"path_trace_depth": 1}, {"light_samples": 1}, {"syn_shadow_samples": 1},
         {"show_nerf": 0}, {"fast_slab": 0}]
for ov in CASES:
    tb, eng, _ = S.make_engine("c3", overrides={"concurrent_streams": 0, "show_nerf": 1, **ov})
    ts = []
    for i in range(4):
        r = eng.frame(collect_kernel_times=True)
        ts.append(r.ms_raytrace)
    d = r.download("syn_depth")
    print(json.dumps({"overrides": ov, "ms_raytrace": round(min(ts[1:]), 3), "hit_px_frac": round(float((d < 100).mean()), 4)}), flush=True)
    tb.close()
