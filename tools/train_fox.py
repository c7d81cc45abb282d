"""Online training on the reference's real fox capture (data/nerf/fox270, tools/make_fox.py) on the GPU box.

The base.json network at the dataset's aabb_scale 4 (per_level_scale 2.438..., 3 cascades, cone stepping 1/256)
from a fresh init, batch 2^18 samples, the dataset's OpenCV lens (k1 k2 p1 p2) and principal point in every
training ray (generate_training_samples_nerf's uv_to_ray(..., lens), testbed_nerf.cu:890-905), every 10th view
held out.  Held-out PSNR renders each held-out view through Testbed::set_camera_to_training_view (its camera,
focal, principal point and lens; render_with_lens_distortion on) with the instant-NGP Shade path at the image's
270x480, sRGB against the image.  Writes the trained model with sng_save_snapshot (the dataset block carries the
lens, so sng_load_snapshot restores render_lens) and reports the step rate, loss and PSNR as one JSON line.

usage: python tools/train_fox.py [steps] [out.ingp]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np

from synerfgine_amd import Engine, Testbed, nerf_data, synthetic

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
OUT = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out", "fox.ingp")
HOLD = 10

d = nerf_data.load_nerf(os.path.join(REPO, "data", "nerf", "fox270"))
imgs, xf, focal, pp, lenses = d["images"], d["xforms"], d["focal"], d["pp"], d["lenses"]
n = len(imgs)
test = list(range(0, n, HOLD))
train = [i for i in range(n) if i not in test]
H, W = imgs.shape[1:3]

tb = Testbed(0)
cfg, params = synthetic.random_init(1337, aabb_scale=d["aabb_scale"])
tb.set_nerf_model(cfg, params)
eng = Engine(tb)
tb.set_training_dataset(imgs[train], xf[train], focal[train], pp[train])
tb.set_training_lens([lenses[i] for i in train])
tb.train_reset(1337)
print(json.dumps({"dataset": "fox270", "aabb_scale": d["aabb_scale"], "per_level_scale": cfg["per_level_scale"], "train_views": len(train),
                  "test_views": test, "res": [W, H], "lens": lenses[0]}), flush=True)

t0 = time.time()
done, hist = 0, []
while done < STEPS:
    k = min(250, STEPS - done)
    st = tb.train(k)
    done += k
    hist.append(st)
    print(json.dumps({**st, "wall_s": round(time.time() - t0, 2)}), flush=True)
wall = time.time() - t0
os.makedirs(os.path.dirname(OUT), exist_ok=True)
tb.save_snapshot(OUT)   # the training dataset's lens goes into the snapshot's dataset block


def to_srgb(rgba):
    lin = np.clip(rgba[..., :3], 0, None)
    return np.clip(np.where(lin < 0.0031308, 12.92 * lin, 1.055 * np.power(lin, 0.41666) - 0.055), 0, 1)


def psnr_of(view_imgs, view_xf, view_focal, view_pp, view_lens, save=None):
    """set_camera_to_training_view needs the views in the training dataset: swap them in (the model is kept)"""
    tb.set_training_dataset(view_imgs, view_xf, view_focal, view_pp)
    tb.set_training_lens(view_lens)
    eng.init(W, H)
    eng.set_param("res_factor", 8)
    out = []
    for k in range(len(view_imgs)):
        tb.set_camera_to_training_view(k)
        rgba = eng.render_nerf(render_mode=1).download("nerf_rgba")
        gt = view_imgs[k].astype(np.float32) / 255.0
        err = np.mean((to_srgb(rgba) - gt[..., :3] * gt[..., 3:4]) ** 2)
        out.append(float(10 * np.log10(1.0 / max(err, 1e-12))))
        if save and k == 0:
            try:
                from PIL import Image
                Image.fromarray((to_srgb(rgba) * 255 + 0.5).astype(np.uint8)).save(save)
            except ImportError:
                pass
    return out


psnrs = psnr_of(imgs[test], xf[test], focal[test], pp[test], [lenses[i] for i in test],
                save=os.path.join(os.path.dirname(OUT), f"fox_view{test[0]}.png"))
few = [train[0], train[len(train) // 2]]
train_psnrs = psnr_of(imgs[few], xf[few], focal[few], pp[few], [lenses[i] for i in few])
# the same held-out views without the lens (Perspective rays through the same pixels): what the lens is worth
persp = psnr_of(imgs[test], xf[test], focal[test], pp[test], [])
ms = [h["ms"] for h in hist[1:]] or [hist[0]["ms"]]
print(json.dumps({"steps": done, "wall_s": round(wall, 2), "steps_per_s": round(done / wall, 1), "ms_per_step_device": round(float(np.mean(ms)) / 250, 3),
                  "final_loss": hist[-1]["loss"], "heldout_psnr": [round(p, 2) for p in psnrs], "heldout_psnr_mean": round(float(np.mean(psnrs)), 2),
                  "heldout_psnr_without_lens_mean": round(float(np.mean(persp)), 2),
                  "train_view_psnr": [round(p, 2) for p in train_psnrs], "density_grid_mean": tb.density_grid_mean(),
                  "ingp": OUT, "ingp_bytes": os.path.getsize(OUT)}), flush=True)
tb.close()
