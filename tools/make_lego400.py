"""Make data/nerf/lego400: the reference's NeRF-synthetic lego training set (data/nerf/lego, 100 x 800^2
RGBA PNG + transforms.json) box-downsampled to 400^2, so it can travel to the GPU box (8.6 MB instead of
42 MB).  The camera poses are unchanged; fl_x/fl_y/cx/cy/w/h are halved.  Run once in the container that
holds /root/reference; the output is committed data (inputs of the BASELINE config-5 training run).
"""
import json
import os
import sys

from PIL import Image

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data/nerf/lego"
DST = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "nerf", "lego400")
S = 400

with open(os.path.join(SRC, "transforms.json")) as f:
    meta = json.load(f)
w0 = meta.get("w", 800)
k = S / w0
os.makedirs(os.path.join(DST, "train"), exist_ok=True)
for key in ("w", "h"):
    if key in meta:
        meta[key] = int(round(meta[key] * k))
for key in ("fl_x", "fl_y", "cx", "cy"):
    if key in meta:
        meta[key] = meta[key] * k
for fr in meta["frames"]:
    p = fr["file_path"]
    src = os.path.join(SRC, p if os.path.splitext(p)[1] else p + ".png")
    rel = os.path.join("train", os.path.basename(src))
    img = Image.open(src).convert("RGBA")
    img.resize((S, S), Image.BOX).save(os.path.join(DST, rel), optimize=True)
    fr["file_path"] = "./" + rel
with open(os.path.join(DST, "transforms.json"), "w") as f:
    json.dump(meta, f, indent=1)
print(f"wrote {len(meta['frames'])} frames to {DST}")
