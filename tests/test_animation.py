"""Scene animation on the host: the camera path (cam_path.cuh:30-143 driving
Testbed::set_view_dir / set_look_at / set_scale, testbed.cu:405-425), light ping-pong motion
(light.cuh:39-49) and object rotation (virtual_object.cuh:53-64), advanced once per Engine::frame
(engine.cu:365-372, 80-127).  libsng_hip.so's host-only sng_animation_probe against the oracle's
restatement, bit for bit (the same float expressions, -ffp-contract=off on both sides)."""
import json
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARMADILLO = os.path.join(REPO, "scenes", "armadillo.json")


def _animated_scene(tmp_path):
    """armadillo.json plus an orbiting object, a second animated light and move_on_start."""
    sc = json.load(open(ARMADILLO))
    sc["camera"]["move_on_start"] = True
    sc["camera"]["animation_speed"] = 0.75
    sc["camera"]["total_time_ms"] = 2000
    sc["objfile"][0]["file"] = os.path.join(REPO, "data", "obj", "armadillo.obj")
    sc["objfile"][0]["anim"] = {"rot_center": [0.5, 0.5, 0.5], "rot_axis": [0.0, 1.0, 0.0], "rot_angle": 0.05}
    sc["lights"][1]["anim"] = {"end": [0.9, 0.2, 1.0], "step": 0.3}
    p = tmp_path / "animated.json"
    p.write_text(json.dumps(sc))
    return str(p), sc


def _compare(path, sc, n, oracle_lib, **kw):
    from synerfgine_amd import animation_probe
    cams, lp, op = animation_probe(path, n, **kw)
    ocams, olp, oop = oracle_lib.animation_play(sc, n, playing=kw.get("playing"), anim_speed=kw.get("animation_speed"))
    np.testing.assert_array_equal(cams, ocams.reshape(n, 4, 3).transpose(0, 2, 1))
    np.testing.assert_array_equal(lp, olp)
    np.testing.assert_array_equal(op, oop)
    return cams, lp, op


def test_camera_path_plays_and_wraps(oracle_lib):
    """armadillo.json's 13-keyframe path: 96 frames at 24 fps over 4 s, 8 frames per segment, wrap to 0."""
    sc = json.load(open(ARMADILLO))
    cams, lp, op = _compare(ARMADILLO, sc, 200, oracle_lib, playing=True)
    look = cams[:, :, 3] + cams[:, :, 2] * 0  # camera positions move along the path
    assert np.abs(np.diff(look, axis=0)).sum() > 0
    # keyframe k is reached exactly every 8 frames (k = frame / 8): view direction equals the normalised keyframe view
    keys = sc["camera"]["path"]
    for f in (8, 16, 40):
        v = np.array(keys[f // 8]["view"], np.float32)
        np.testing.assert_allclose(cams[f - 1][:, 2], v / np.linalg.norm(v), atol=1e-6)
    # no animation_speed in armadillo.json: lights and objects do not move
    assert (lp == lp[0]).all() and (op == op[0]).all()


def test_not_playing_keeps_camera(oracle_lib):
    sc = json.load(open(ARMADILLO))
    cams, _, _ = _compare(ARMADILLO, sc, 5, oracle_lib)
    assert (cams == cams[0]).all()


def test_objects_and_lights_animate(tmp_path, oracle_lib):
    path, sc = _animated_scene(tmp_path)
    cams, lp, op = _compare(path, sc, 60, oracle_lib)
    assert np.abs(np.diff(op[:, 0], axis=0)).max() > 0          # the object moves
    # the animated light bounces between its start and end (step 0.3: ratio 0.3, 0.6, 0.9, then back)
    start, end = np.array(sc["lights"][1]["pos"], np.float32), np.array([0.9, 0.2, 1.0], np.float32)
    ratios = [(p - start)[0] / (end - start)[0] for p in lp[:8, 1]]
    np.testing.assert_allclose(ratios, [0.3, 0.6, 0.9, 0.6, 0.3, 0.0, 0.3, 0.6], atol=1e-5)


def test_probe_rejects_bad_scene(tmp_path):
    from synerfgine_amd import SngError, animation_probe
    sc = json.load(open(ARMADILLO))
    del sc["camera"]["total_time_ms"]
    p = tmp_path / "bad.json"
    p.write_text(json.dumps(sc))
    with pytest.raises(SngError):
        animation_probe(str(p), 3)
