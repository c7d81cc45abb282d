"""`.ingp` snapshot writer: zlib(msgpack) with the keys Testbed::load_snapshot reads
(testbed.cu:4812-4876 save, 4878-5015 load).

Host tooling: turns the synthetic snapshot content (synthetic.py) into a real file so the
product's loader (sng_load_snapshot / sng_snapshot_probe) is exercised end to end.  Written
tcnn fields: params_binary (+ params_type "__half", n_params), density_grid_binary (fp16,
128^3 x (max_cascade+1)), density_grid_size, nerf.aabb_scale, camera {matrix, fov_axis,
relative_focal_length, screen_center, zoom, scale}, version 1, and the encoding config.
"""
import zlib

import numpy as np


def write_ingp(path, cfg, params_f16, grid_f16, camera=None, aabb_scale=None):
    import msgpack
    params = np.ascontiguousarray(params_f16, np.float16)
    grid = np.ascontiguousarray(grid_f16, np.float16)
    a = int(aabb_scale if aabb_scale is not None else cfg.get("aabb_scale", 1))
    snap = {
        "version": 1,
        "mode": "nerf",
        "params_type": "__half",
        "n_params": int(params.size),
        "params_binary": params.tobytes(),
        "density_grid_size": 128,
        "density_grid_binary": grid.tobytes(),
        "nerf": {"aabb_scale": a, "dataset": {"aabb_scale": a}},
    }
    if camera is not None:
        snap["camera"] = camera
    root = {
        "snapshot": snap,
        "encoding": {"otype": "HashGrid", "n_levels": int(cfg["n_levels"]), "n_features_per_level": int(cfg["n_features_per_level"]),
                     "log2_hashmap_size": int(cfg["log2_hashmap_size"]), "base_resolution": int(cfg["base_resolution"]),
                     "per_level_scale": float(cfg["per_level_scale"])},
        "network": {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 64, "n_hidden_layers": 1},
        "dir_encoding": {"otype": "SphericalHarmonics", "degree": 4},
        "rgb_network": {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 64, "n_hidden_layers": 2},
    }
    with open(path, "wb") as f:
        f.write(zlib.compress(msgpack.packb(root, use_bin_type=True), 6))


def read_ingp(path):
    """Host-side read of an .ingp (zlib(msgpack) or plain msgpack) -> (cfg, params fp16, density grid fp16).
    Data only (msgpack decodes no code); the product's loader is sng_load_snapshot -- this reader feeds the
    oracle and the tests the same model content."""
    import msgpack
    with open(path, "rb") as f:
        raw = f.read()
    try:
        raw = zlib.decompress(raw, 47)   # 32 + 15: zlib or gzip wrapper (zstr writes gzip), as the C++ loader's inflateInit2(15 + 32)
    except zlib.error:
        pass
    root = msgpack.unpackb(raw, raw=False, strict_map_key=False)
    snap, enc = root["snapshot"], root["encoding"]
    if snap.get("params_type", "__half") != "__half":
        params = np.frombuffer(snap["params_binary"], np.float32).astype(np.float16)
    else:
        params = np.frombuffer(snap["params_binary"], np.float16).copy()
    grid = np.frombuffer(snap["density_grid_binary"], np.float16).copy()
    nerf = snap.get("nerf", {})
    a = nerf.get("aabb_scale", nerf.get("dataset", {}).get("aabb_scale", 1))
    cfg = dict(n_levels=int(enc["n_levels"]), n_features_per_level=int(enc["n_features_per_level"]),
               log2_hashmap_size=int(enc["log2_hashmap_size"]), base_resolution=int(enc["base_resolution"]),
               per_level_scale=float(enc["per_level_scale"]), aabb_scale=int(a))
    return cfg, params, grid
