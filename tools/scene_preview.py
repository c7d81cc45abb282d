"""Render one frame of a workload config (synerfgine_amd.scene.CONFIGS) at a small size and save it as a PNG, with
the frame's march statistics (samples per pixel, iterations, one-step regime) -- for placing a scene's camera,
lights and objects (scenes/fox-rocks.json) before benchmarking it.

usage: python tools/scene_preview.py CONFIG MODEL WIDTH HEIGHT OUT.png [KEY=VALUE ...]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np

from synerfgine_amd import scene as S

config, model, w, h, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
ov = {kv.split("=")[0]: float(kv.split("=")[1]) for kv in sys.argv[6:]}
tb, eng, _ = S.make_engine(config, width=w, height=h, model=model, overrides=ov)
eng.frame(spp=0, reset=True)
r = eng.frame(spp=0, reset=True, collect_kernel_times=True)
rgb = np.clip(r.download("final_rgba")[..., :3], 0, 1)
from PIL import Image
Image.fromarray((rgb * 255 + 0.5).astype(np.uint8)).save(out)
px = w * h
print(json.dumps({"config": config, "res": [w, h], "ms_frame": r.ms_frame, "samples_per_px": r.n_samples / px, "hit_frac": r.n_hit / px,
                  "iterations": r.n_iterations, "onestep": [r.onestep_from_iter, r.onestep_iterations], "msr_rounds": r.msr_rounds,
                  "stages": {"raytrace": r.ms_raytrace, "nerf": r.ms_nerf, "shadow": r.ms_shadow}}))
tb.close()
