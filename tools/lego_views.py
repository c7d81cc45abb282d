"""Probe camera views of the lego snapshot (NeRF only): hit fraction and samples per hit ray per view.
usage (GPU box): python tools/lego_views.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from synerfgine_amd import scene as S  # noqa: E402

VIEWS = [((0.62, 0.46, -0.64), 0.9), ((0.62, 0.46, -0.64), 1.2), ((0.62, -0.46, -0.64), 0.9), ((0.62, -0.46, -0.64), 1.2),
         ((-0.6, 0.5, 0.6), 1.0), ((-0.6, -0.5, 0.6), 1.0), ((0.0, 0.0, -1.0), 1.0), ((0.0, -1.0, 0.0), 1.0), ((0.0, 1.0, 0.0), 1.0)]
tb, eng, _ = S.make_engine("c2", width=400, height=400, model="lego")
for v, s in VIEWS:
    tb.set_camera_view(v, (0.5, 0.5, 0.5), s)
    r = eng.frame()
    print(json.dumps({"view": v, "scale": s, "hit_frac": round(r.n_hit / 160000, 3), "samples_per_hit": round(r.n_samples / max(1, r.n_hit), 1),
                      "iters": r.n_iterations}), flush=True)
tb.close()
