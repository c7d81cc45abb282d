"""Workload setup shared by bench.py, smoke() and the tests (no oracle imports here)."""
import os

import numpy as np

from . import Engine, Testbed
from . import synthetic

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(REPO, "scenes")

# BASELINE.json configs: C2 = lego only 800x800; C3 = lego + armadillo 1920x1080 with shadows
CONFIGS = {
    "c2": dict(scene="armadillo.json", width=800, height=800, overrides={"show_virtual_obj": 0, "shadow_on_nerf": 0,
                                                                            "shadow_on_virtual_obj": 0}),
    "c3": dict(scene="armadillo.json", width=1920, height=1080, overrides={}),
    "c4": dict(scene="kitchen-rocks.json", width=1920, height=1080, overrides={"light_samples": 4}),
}

_MODEL_CACHE = {}


def model_for(config, seed=1337):
    """Synthetic snapshot content of a config (cached per process): lego-like or kitchen-like."""
    key = ("kitchen" if config == "c4" else "lego", seed)
    if key not in _MODEL_CACHE:
        _MODEL_CACHE[key] = synthetic.kitchen_like(seed=seed) if config == "c4" else synthetic.lego_like(seed=seed)
    return _MODEL_CACHE[key]


def make_engine(config="c3", device_id=0, width=None, height=None, overrides=None, seed=1337):
    """Testbed with the synthetic lego-like snapshot + Engine with the config's scene JSON."""
    cfg = CONFIGS[config]
    tb = Testbed(device_id)
    ncfg, params, grid = model_for(config, seed)
    tb.set_nerf_model(ncfg, params)
    tb.set_density_grid(grid)
    eng = Engine(tb)
    eng.set_virtual_world(os.path.join(SCENES, cfg["scene"]))
    for k, v in {**cfg["overrides"], **(overrides or {})}.items():
        eng.set_param(k, v)
    eng.init(width or cfg["width"], height or cfg["height"])
    return tb, eng, (ncfg, params, grid)
