"""Workload setup shared by bench.py, smoke() and the tests (no oracle imports here)."""
import os

import numpy as np

from . import Engine, Testbed
from . import ingp, synthetic

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(REPO, "scenes")

# BASELINE.json configs: C2 = lego only 800x800; C3 = lego + armadillo 1920x1080 with shadows
CONFIGS = {
    "c2": dict(scene="armadillo.json", width=800, height=800, overrides={"show_virtual_obj": 0, "shadow_on_nerf": 0,
                                                                            "shadow_on_virtual_obj": 0}),
    "c3": dict(scene="armadillo.json", width=1920, height=1080, overrides={}),
    "c4": dict(scene="kitchen-rocks.json", width=1920, height=1080, overrides={"light_samples": 4}),
    # C4's workload (bunny / rock / box, one light, light_samples 4, NeRF shadows r = 2) on a TRAINED cascaded field:
    # the reference's real fox capture (aabb_scale 4, OpenCV lens) trained by tools/train_fox.py, camera and object
    # placement of scenes/fox-rocks.json (kitchen-rocks.json's rendering block, materials and meshes)
    "c4fox": dict(scene="fox-rocks.json", width=1920, height=1080, overrides={"light_samples": 4}),
    # the reference's own scene for the fox capture (scripts/virtual_desc/fox-armadillo.json, copied unmodified): its
    # camera in the fox frame, a point light + a directional light, bunny + armadillo, nerf_on_nerf_shadow_threshold
    # 0.942, light_samples 8 -- rendered on the trained fox snapshot
    "foxarm": dict(scene="fox-armadillo.json", width=1920, height=1080, overrides={}),
    # the scene of every reference measurement in BASELINE.md (scripts/render/profiling.sh:12-18): lego +
    # armadillo/bunny/monkey at 1280x720, swept over --sshadows/--nshadows in {1,2,4,8}
    "abm": dict(scene="dmrf-compare-abm.json", width=1280, height=720, overrides={}),
}

# the trained lego snapshot (tools/train_lego.py on data/nerf/lego400, the reference's lego set); configs
# c2/c3 render it when model="lego" (bench.py's default), the tests default to the synthetic model
LEGO_INGP = os.path.join(REPO, "data", "lego.ingp")
# the trained fox snapshot (tools/train_fox.py on data/nerf/fox270, the reference's fox capture); config c4fox
FOX_INGP = os.path.join(REPO, "data", "fox.ingp")

FOX_CONFIGS = ("c4fox", "foxarm")

_MODEL_CACHE = {}


def snapshot_path(config, model):
    """.ingp path a (config, model) pair renders, or None for the synthetic content."""
    if model in (None, "synthetic"):
        if config in FOX_CONFIGS:
            raise ValueError(f"{config} renders the trained fox snapshot (data/fox.ingp)")
        return None
    if model == "fox" or (config in FOX_CONFIGS and model in ("lego", "default")):
        return FOX_INGP
    if model == "lego":
        if config == "c4":
            raise ValueError("c4 renders the kitchen-like synthetic snapshot (no kitchen capture in the reference)")
        return LEGO_INGP
    return model


def model_for(config, seed=1337, model="synthetic"):
    """Snapshot content of a config (cached per process): the synthetic lego-like / kitchen-like model, or
    (cfg, params, grid) read from an .ingp (model="lego" or a path)."""
    path = snapshot_path(config, model)
    key = (path,) if path else ("kitchen" if config == "c4" else "lego", seed)
    if key not in _MODEL_CACHE:
        if path:
            _MODEL_CACHE[key] = ingp.read_ingp(path)
        else:
            _MODEL_CACHE[key] = synthetic.kitchen_like(seed=seed) if config == "c4" else synthetic.lego_like(seed=seed)
    return _MODEL_CACHE[key]


def make_engine(config="c3", device_id=0, width=None, height=None, overrides=None, seed=1337, model="synthetic"):
    """Testbed with the config's snapshot + Engine with the config's scene JSON.  model="synthetic" sets the
    synthetic model from memory; model="lego" (or an .ingp path) goes through Testbed::load_snapshot."""
    cfg = CONFIGS[config]
    tb = Testbed(device_id)
    path = snapshot_path(config, model)
    ncfg, params, grid = model_for(config, seed, model)
    if path:
        tb.load_snapshot(path)
    else:
        tb.set_nerf_model(ncfg, params)
        tb.set_density_grid(grid)
    eng = Engine(tb)
    eng.set_virtual_world(os.path.join(SCENES, cfg["scene"]))
    # the workloads render a fixed camera (the scene's initial view): kitchen-rocks.json's move_on_start
    # would otherwise advance its camera path on every frame (set camera_path_playing=1 to play it)
    eng.set_param("camera_path_playing", 0)
    for k, v in {**cfg["overrides"], **(overrides or {})}.items():
        eng.set_param(k, v)
    eng.init(width or cfg["width"], height or cfg["height"])
    return tb, eng, (ncfg, params, grid)
