"""Online training smoke / convergence run on a synthetic dataset (GPU box)."""
import json
import sys
import time

sys.path.insert(0, "/root/repo")
import numpy as np

from synerfgine_amd import Engine, Testbed, nerf_data, synthetic

W = H = int(sys.argv[1]) if len(sys.argv) > 1 else 128
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 200
BATCH = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 16
# ground truth: the lego-like analytic model rendered from 24 orbit cameras (+1 held out)
gt_cfg, gt_params, gt_grid = synthetic.lego_like()
tb = Testbed(0)
tb.set_nerf_model(gt_cfg, gt_params)
tb.set_density_grid(gt_grid)
eng = Engine(tb)
cams = nerf_data.orbit_cameras(25)
imgs, xf, focal, pp = nerf_data.render_views(tb, eng, cams, W, H)
print(json.dumps({"dataset": list(imgs.shape), "alpha_cover": float((imgs[..., 3] > 0).mean())}), flush=True)
# fresh network, train
cfg, params = synthetic.random_init(7)
tb.set_nerf_model(cfg, params)
eng.set_param("train_batch", BATCH)
tb.set_training_dataset(imgs[:24], xf[:24], focal[:24], pp[:24])
tb.train_reset(1337)
t0 = time.time()
done = 0
while done < STEPS:
    k = min(50, STEPS - done)
    st = tb.train(k)
    done += k
    print(json.dumps({**st, "wall_s": round(time.time() - t0, 2)}), flush=True)


def psnr(a, b):
    return float(10 * np.log10(1.0 / max(np.mean((a - b) ** 2), 1e-12)))


# held-out view: render the trained model and compare composited-on-black sRGB
tb.camera_matrix = xf[24].T.reshape(-1)
r = eng.render_nerf(render_mode=1)
rgba = r.download("nerf_rgba")
lin = np.clip(rgba[..., :3], 0, None)
pred = np.where(lin < 0.0031308, 12.92 * lin, 1.055 * np.power(lin, 0.41666) - 0.055)
gt = imgs[24].astype(np.float32) / 255.0
gt_rgb = gt[..., :3] * gt[..., 3:4]
print(json.dumps({"heldout_psnr": round(psnr(np.clip(pred, 0, 1), gt_rgb), 2), "steps": done}), flush=True)
tb.close()
