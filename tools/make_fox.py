"""Make data/nerf/fox270: the reference's real-capture fox set (data/nerf/fox: transforms.json with OpenCV lens
k1 k2 p1 p2, principal point cx cy, aabb_scale 4, 67 frames of which 50 have an image, 1080x1920 JPEGs) box-
downsampled by 4 to 270x480 PNGs, so it can travel to the GPU box (the dataset loader decodes PNG only).

Only what the loader reads is rescaled: w, h, fl_x, fl_y, cx, cy (pixel units) by 1/4; the lens coefficients act
on normalised camera coordinates and the poses are unchanged.  Frames whose image is missing are kept in the JSON:
the reference's loader drops them itself (nerf_loader.cu:364-386, the sharpness branch keeps a frame only when its
file exists), and so does synerfgine_amd.nerf_data.load_nerf.  Run once in the container that holds
/root/reference; the output is committed data (inputs of the fox training run, tools/train_fox.py).
"""
import json
import os
import sys

from PIL import Image

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data/nerf/fox"
DST = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "nerf", "fox270")
K = 4

with open(os.path.join(SRC, "transforms.json")) as f:
    meta = json.load(f)
W0, H0 = int(meta["w"]), int(meta["h"])
W, H = W0 // K, H0 // K
assert W * K == W0 and H * K == H0
meta["w"], meta["h"] = float(W), float(H)
for key in ("fl_x", "fl_y", "cx", "cy"):
    meta[key] = meta[key] / K
os.makedirs(os.path.join(DST, "images"), exist_ok=True)
n = 0
for fr in meta["frames"]:
    src = os.path.join(SRC, fr["file_path"])
    stem = os.path.splitext(os.path.basename(src))[0]
    fr["file_path"] = "images/" + stem + ".png"
    if not os.path.exists(src):
        continue
    img = Image.open(src).convert("RGB")
    assert img.size == (W0, H0), img.size
    img.resize((W, H), Image.BOX).save(os.path.join(DST, fr["file_path"]), optimize=True)
    n += 1
with open(os.path.join(DST, "transforms.json"), "w") as f:
    json.dump(meta, f, indent=1)
print(f"wrote {n} of {len(meta['frames'])} frames ({W}x{H}) to {DST}")
