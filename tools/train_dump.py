"""Dump one training step's device buffers (GPU box) for the CPU-side reference check
(tests/train_ref.py): a small lego400 subset, a briefly trained model, then train_nerf_step up to the
gradients with the parity hook.  usage: python tools/train_dump.py [warm_steps] [out.npz]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np

from synerfgine_amd import Engine, Testbed, nerf_data, synthetic

WARM = int(sys.argv[1]) if len(sys.argv) > 1 else 200
OUT = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out", "train_dump.npz")
imgs, xf, focal, pp = nerf_data.load_nerf_synthetic(os.path.join(REPO, "data", "nerf", "lego400"), max_images=16)
tb = Testbed(0)
cfg, params = synthetic.random_init(1337)
tb.set_nerf_model(cfg, params)
eng = Engine(tb)
eng.set_param("train_batch", 1 << 14)
tb.set_training_dataset(imgs, xf, focal, pp)
tb.train_reset(1337)
if WARM:
    print(tb.train(WARM), flush=True)
ctrl = tb.train_debug(4, "ctrl", np.uint32)[:4].copy()
out = {"ctrl": ctrl, "density_mean": np.float32(tb.density_grid_mean())}
nr, ns = int(ctrl[0]), int(min(ctrl[1], 1 << 18))
out["ray_indices"] = tb.train_debug(0, "ray_indices", np.uint32)[:nr]
out["rays"] = tb.train_debug(0, "rays", np.float32)[: 8 * nr]
out["numsteps"] = tb.train_debug(0, "numsteps", np.uint32)[: 2 * nr]
out["coords"] = tb.train_debug(0, "coords", np.float32)[: 7 * ns]
out["mlp_out"] = tb.train_debug(0, "mlp_out", np.uint16)[: 4 * ns]
tgt = 1 << 14
out["coords_c"] = tb.train_debug(0, "coords_c", np.float32)[: 7 * tgt]
out["dloss"] = tb.train_debug(0, "dloss", np.uint16)[: 4 * tgt]
out["loss"] = tb.train_debug(0, "loss", np.float32)[:nr]
g = tb.train_debug(0, "grads", np.float32)
nz = np.nonzero(g)[0].astype(np.uint32)
out["grad_idx"], out["grad_val"] = nz, g[nz]
out["params_train"] = tb.train_debug(0, "master", np.float32).astype(np.float16)
acts = tb.train_debug(0, "acts", np.uint16)
out["acts"] = acts[: (tgt // 16) * 480 * 16]
out["images"], out["xforms"], out["focal"], out["pp"] = imgs, xf, focal, pp
print({k: getattr(v, "shape", v) for k, v in out.items()}, flush=True)
os.makedirs(os.path.dirname(OUT), exist_ok=True)
np.savez_compressed(OUT, **out)
print("wrote", OUT, os.path.getsize(OUT), flush=True)
tb.close()
