"""The CPU oracle reproduces the committed golden fixtures exactly (tests/golden/make_golden.py)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as G  # noqa: E402


def _load(name):
    return dict(np.load(os.path.join(HERE, "golden", name + ".npz")))


@pytest.mark.parametrize("name", ["rng", "encode_l8f4", "encode_l16f2", "bitfield_lego_like", "bvh_armadillo", "frame_nerf_64"])
def test_oracle_reproduces_fixture(name):
    want = _load(name)
    got = G.GENERATORS[name]()
    assert set(got) == set(want)
    for k in want:
        a, b = np.asarray(got[k]), want[k]
        assert a.shape == b.shape, k
        if a.dtype.kind == "f":
            assert np.array_equal(a.view(np.uint32 if a.dtype == np.float32 else np.uint64), b.view(a.view(np.uint32 if a.dtype == np.float32 else np.uint64).dtype)), k
        else:
            assert np.array_equal(a, b), k


def test_bvh_fixture_hits_are_consistent():
    f = _load("bvh_armadillo")
    hit = f["t"] < 1e4
    assert 0.2 < hit.mean() < 0.9
    assert (f["obj"][hit] == 0).all() and (f["obj"][~hit] == -1).all()


def test_frame_fixture_schedule():
    f = _load("frame_nerf_64")
    assert f["n_hit"] > 0 and f["n_samples"] > 0
    assert (f["steps_per_iter"] == 8).all()            # 2^21 / n_alive > 8 at this size
    assert np.all(np.diff(f["alive_per_iter"]) <= 0)
