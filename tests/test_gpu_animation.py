"""GPU: an animated scene (camera path playing, orbiting object, moving light) renders through
sng_render_frame, which advances the animation once per frame like Engine::frame (engine.cu:365-372);
the 4th frame is compared with the CPU oracle given that frame's state, and the state itself with
the host-only probe (bit-exact, tests/test_animation.py covers the probe against the oracle)."""
import json
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.oracle_mode("literal")]   # the oracle compares the reference's text as written
torch = pytest.importorskip("torch")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_animated_frames_match_oracle(tmp_path, synthetic_model, oracle_lib):
    from synerfgine_amd import animation_probe
    from synerfgine_amd import scene as S
    O = oracle_lib
    sc = json.load(open(os.path.join(REPO, "scenes", "armadillo.json")))
    sc["camera"]["move_on_start"] = True
    sc["camera"]["animation_speed"] = 1.0
    sc["objfile"][0]["file"] = os.path.join(REPO, "data", "obj", "armadillo.obj")
    sc["objfile"][0]["anim"] = {"rot_center": [0.5, 0.5, 0.5], "rot_axis": [0.0, 1.0, 0.0], "rot_angle": 0.1}
    path = tmp_path / "anim.json"
    path.write_text(json.dumps(sc))
    tb, eng, (ncfg, params, grid) = S.make_engine("c3", width=96, height=54, overrides={"res_factor": 8})
    eng.set_virtual_world(str(path))
    eng.init(96, 54)
    cams, lp, op = animation_probe(str(path), 4)
    frames = []
    for f in range(3):
        frames.append(eng.frame(spp=0, reset=True).download("final_rgba").copy())
    nrng, mrng = eng.rng_states(0).copy(), eng.rng_states(1).copy()
    gpu = eng.frame(spp=0, reset=True).download("final_rgba")
    objs, lights, _ = eng.scene()
    np.testing.assert_array_equal(objs[0]["pos"], op[3, 0])
    np.testing.assert_array_equal(np.array(lights[0]["pos"], np.float32), lp[3, 0])
    np.testing.assert_array_equal(np.asarray(tb.camera_matrix, np.float32).reshape(4, 3).T, cams[3])
    assert not np.array_equal(frames[0], frames[2]), "animation had no visible effect"
    ref = O.render_frame(O.Model(ncfg, params), O.make_volume(O.bitfield(grid)[0]), tb, eng, nrng, mrng)
    tb.close()
    err = np.abs(np.clip(gpu[..., :3], 0, 1) - np.clip(ref["final"][..., :3], 0, 1))
    psnr = 10 * np.log10(1.0 / max(float(np.mean(err ** 2)), 1e-12))
    assert psnr >= 40.0 and (err.max(axis=-1) <= 2 / 255).mean() >= 0.995, (psnr, float(err.max()))
