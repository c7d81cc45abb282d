"""Training-path diagnostics: device weight packing vs host packing, render/GT comparison math."""
import json
import sys

sys.path.insert(0, "/root/repo")
import numpy as np

from synerfgine_amd import Engine, Testbed, nerf_data, synthetic

W = H = 128
gt_cfg, gt_params, gt_grid = synthetic.lego_like()
tb = Testbed(0)
tb.set_nerf_model(gt_cfg, gt_params)
tb.set_density_grid(gt_grid)
eng = Engine(tb)
cams = nerf_data.orbit_cameras(25)
imgs, xf, focal, pp = nerf_data.render_views(tb, eng, cams, W, H)


def render(i):
    tb.camera_matrix = xf[i].T.reshape(-1)
    r = eng.render_nerf(render_mode=1)
    return r.download("nerf_rgba")


def to_srgb(rgba):
    lin = np.clip(rgba[..., :3], 0, None)
    return np.clip(np.where(lin < 0.0031308, 12.92 * lin, 1.055 * np.power(lin, 0.41666) - 0.055), 0, 1)


def psnr(a, b):
    return float(10 * np.log10(1.0 / max(np.mean((a - b) ** 2), 1e-12)))


A = render(24)
gt = imgs[24].astype(np.float32) / 255.0
print(json.dumps({"gt_vs_render_psnr": psnr(to_srgb(A), gt[..., :3] * gt[..., 3:4])}), flush=True)
tb.set_training_dataset(imgs[:24], xf[:24], focal[:24], pp[:24])
tb.train_reset(1337)
tb.train(0)
B = render(24)
print(json.dumps({"repacked_equal": bool(np.array_equal(A, B)), "max_diff": float(np.abs(A - B).max())}), flush=True)
# one stage at a time
for stage, name, dt in [(1, "ctrl", np.uint32), (2, "mlp_out", np.float16), (3, "dloss", np.float16), (4, "grads", np.float32)]:
    v = tb.train_debug(stage, name, dt)
    if name == "ctrl":
        print(json.dumps({"ctrl": v[:4].tolist()}), flush=True)
    else:
        f = v.astype(np.float32)
        print(json.dumps({name: {"nonzero": int((f != 0).sum()), "absmax": float(np.abs(f).max()), "nan": int(np.isnan(f).sum())}}), flush=True)
ri = tb.train_debug(1, "ray_indices", np.uint32)
ctrl = tb.train_debug(0, "ctrl", np.uint32)
n = int(ctrl[0])
idx = ri[:n]
print(json.dumps({"n_rays_hit": n, "images": sorted(set((idx * 24 // 4096).tolist())), "first_idx": idx[:10].tolist()}), flush=True)
rays = tb.train_debug(0, "rays", np.float32)[: 8 * n].reshape(n, 8)
print(json.dumps({"ray0": rays[0].tolist() if n else None, "cam0": xf[int(idx[0]) * 24 // 4096].tolist() if n else None}), flush=True)
eng.set_param("train_debug", 1)
js = tb.train_debug(1, "loss", np.float32)[:4096]
tt = tb.train_debug(0, "coords_c", np.float32)[:8192].reshape(4096, 2)
print(json.dumps({"rays_j_gt0": int((js > 0).sum()), "tmin_finite": int((tt[:, 0] < 1e30).sum()), "tmin_sample": tt[:5, 0].tolist(),
                  "startt_sample": tt[:5, 1].tolist(), "j_sample": js[:20].tolist()}), flush=True)
g = tb.train_debug(0, "grads", np.float32)
print(json.dumps({"grad_mlp_absmax": float(np.abs(g[:10240]).max()), "grad_mlp_nz": int((g[:10240] != 0).sum()),
                  "grad_grid_absmax": float(np.abs(g[10240:]).max()), "grad_grid_nz": int((g[10240:] != 0).sum())}), flush=True)
tb.close()
