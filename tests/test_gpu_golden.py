"""HIP path (through the C-ABI) against the committed golden fixtures (tests/golden/*.npz)."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as G  # noqa: E402


def _load(name):
    return dict(np.load(os.path.join(HERE, "golden", name + ".npz")))


def _fp16_ulp(x):
    x = np.abs(np.asarray(x, np.float32))
    return np.exp2(np.floor(np.log2(np.maximum(x, 6.1e-5))) - 10)


@pytest.mark.parametrize("name,cfg", [("encode_l8f4", G.L8F4), ("encode_l16f2", G.L16F2)])
def test_encode_matches_fixture(name, cfg):
    from synerfgine_amd import Testbed
    f = _load(name)
    tb = Testbed(0)
    try:
        tb.set_nerf_model(cfg, G.random_params(cfg))
        c = f["coords"]
        n = c.shape[0]
        dc = torch.from_numpy(c).cuda()
        width = cfg["n_levels"] * cfg["n_features_per_level"]
        out = torch.zeros((n, 32), dtype=torch.float16, device="cuda")
        tb.encode(dc.data_ptr(), 7, n, out.data_ptr())
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint16)[:, :width]
        assert np.array_equal(got, f["encoding"][:, :width])
        if "network" in f:
            o = torch.zeros((512, 4), dtype=torch.float16, device="cuda")
            tb.inference_mixed_precision(dc.data_ptr(), 7, 512, o.data_ptr(), layout=1)
            torch.cuda.synchronize()
            g = o.cpu().numpy().astype(np.float32)
            e = f["network"].view(np.float16).astype(np.float32)[:, :4]
            assert (np.abs(g - e) <= 2 * _fp16_ulp(e) + 1e-3).all()
    finally:
        tb.close()


def test_bitfield_and_rng_match_fixtures(synthetic_model):
    import hashlib
    from synerfgine_amd import scene as S
    bf = _load("bitfield_lego_like")
    rng = _load("rng")
    tb, eng, _ = S.make_engine("c2", width=64, height=64, overrides={"res_factor": 8})
    try:
        b = tb.density_grid_bitfield()
        assert np.array_equal(np.frombuffer(hashlib.sha256(b.tobytes()).digest(), np.uint8), bf["sha256"])
        assert tb.density_grid_mean() == float(bf["mean"])
        st = eng.rng_states(0)
        assert np.array_equal(st[:4096], rng["xorwow_states"])
    finally:
        tb.close()


def test_nerf_frame_matches_fixture():
    from synerfgine_amd import scene as S
    f = _load("frame_nerf_64")
    tb, eng, _ = S.make_engine("c2", width=64, height=64, overrides={"res_factor": 8})
    try:
        tb.camera_matrix = f["camera"]
        foc = tb.focal_length(0)
        assert abs(foc[1] - float(f["focal"])) <= 1e-5 * float(f["focal"])
        r = eng.frame()
        got = r.download("nerf_rgba")
        n = min(len(r.alive_per_iter), len(f["alive_per_iter"]))
        assert abs(r.n_iterations - int(f["n_iterations"])) <= 1
        assert np.allclose(r.alive_per_iter[:n], f["alive_per_iter"][:n], rtol=0.01, atol=2)
        mse = float(np.mean((np.clip(got[..., :3], 0, 1) - np.clip(f["rgba"][..., :3], 0, 1)) ** 2))
        assert 10 * np.log10(1.0 / max(mse, 1e-12)) >= 40.0
    finally:
        tb.close()
