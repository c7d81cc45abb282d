"""Online training on the reference's lego set (BASELINE config 5) on the GPU box.

Trains the base.json network (L=8, F=4, T=2^19, 64-wide density/rgb MLPs) from a fresh init on
data/nerf/lego400 (tools/make_lego400.py) with the reference's defaults (batch 2^18 samples,
Ema(ExpDecay(Adam)), density-grid EMA every 16 steps), holds out every 20th view, and reports
training throughput, loss and held-out PSNR.  Writes the trained model as an .ingp snapshot.

usage: [SNG_SET=key=value,...] [FOCAL_FROM_ANGLE=1] python tools/train_lego.py [steps] [out.ingp]
"""
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np

from synerfgine_amd import Engine, Testbed, ingp, nerf_data, synthetic

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
OUT = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out", "lego.ingp")
HOLD = 20

imgs, xf, focal, pp = nerf_data.load_nerf_synthetic(os.path.join(REPO, "data", "nerf", "lego400"))
if os.environ.get("FOCAL_FROM_ANGLE"):
    # transforms.json carries fl_x = 1000 (@800 px) beside camera_angle_x = 0.6911 (-> 1111 px, the
    # Blender render's focal); ngp's read_focal_length (nerf_loader.cu:243-270) prefers fl_x
    angle = json.load(open(os.path.join(REPO, "data", "nerf", "lego400", "transforms.json")))["camera_angle_x"]
    focal[:] = 0.5 * imgs.shape[2] / math.tan(0.5 * angle)
n = len(imgs)
test = list(range(0, n, HOLD))
train = [i for i in range(n) if i not in test]
H, W = imgs.shape[1:3]

tb = Testbed(0)
cfg, params = synthetic.random_init(1337)
tb.set_nerf_model(cfg, params)
eng = Engine(tb)
for kv in filter(None, os.environ.get("SNG_SET", "").split(",")):   # engine parameters, e.g. SNG_SET=train_grid_grad_f16=1
    eng.set_param(kv.split("=")[0], float(kv.split("=")[1]))
tb.set_training_dataset(imgs[train], xf[train], focal[train], pp[train])
tb.train_reset(1337)
print(json.dumps({"dataset": "lego400", "train_views": len(train), "test_views": test, "res": [W, H]}), flush=True)

t0 = time.time()
done, hist = 0, []
while done < STEPS:
    k = min(250, STEPS - done)
    st = tb.train(k)
    done += k
    hist.append(st)
    print(json.dumps({**st, "wall_s": round(time.time() - t0, 2)}), flush=True)
wall = time.time() - t0


def to_srgb(rgba):
    lin = np.clip(rgba[..., :3], 0, None)
    return np.clip(np.where(lin < 0.0031308, 12.92 * lin, 1.055 * np.power(lin, 0.41666) - 0.055), 0, 1)


eng.init(W, H)
eng.set_param("res_factor", 8)
tb.set_fov(math.degrees(2.0 * math.atan(0.5 * H / float(focal[0][1]))))
psnrs, train_psnrs = [], []
for i in test + [train[0], train[len(train) // 2]]:
    tb.camera_matrix = np.asarray(xf[i], np.float32).T.reshape(-1)
    rgba = eng.render_nerf(render_mode=1).download("nerf_rgba")
    gt = imgs[i].astype(np.float32) / 255.0
    err = np.mean((to_srgb(rgba) - gt[..., :3] * gt[..., 3:4]) ** 2)
    (psnrs if i in test else train_psnrs).append(float(10 * np.log10(1.0 / max(err, 1e-12))))
    if i == test[0]:
        try:
            from PIL import Image
            os.makedirs(os.path.dirname(OUT), exist_ok=True)
            Image.fromarray((to_srgb(rgba) * 255 + 0.5).astype(np.uint8)).save(os.path.join(os.path.dirname(OUT), f"lego_view{i}.png"))
        except ImportError:
            pass

p16, g16 = tb.training_snapshot(synthetic.n_params(), 128 ** 3)
os.makedirs(os.path.dirname(OUT), exist_ok=True)
ingp.write_ingp(OUT, cfg, p16, g16, aabb_scale=1)
ms = [h["ms"] for h in hist[1:]] or [hist[0]["ms"]]
print(json.dumps({"steps": done, "wall_s": round(wall, 2), "steps_per_s": round(done / wall, 1), "ms_per_step_device": round(float(np.mean(ms)) / 250, 3),
                  "final_loss": hist[-1]["loss"], "heldout_psnr": [round(p, 2) for p in psnrs], "heldout_psnr_mean": round(float(np.mean(psnrs)), 2),
                  "train_view_psnr": [round(p, 2) for p in train_psnrs],
                  "density_grid_mean": tb.density_grid_mean(), "ingp": OUT, "ingp_bytes": os.path.getsize(OUT)}), flush=True)
tb.close()
