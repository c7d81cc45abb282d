"""GPU parity of the lens models (SURVEY.md §8(f) rank 1 on the reference's real fox capture; VERDICT r04
"missing" 1-2) through the C ABI, against the CPU oracle:

  * training samples of the fox set (data/nerf/fox270: OpenCV k1 k2 p1 p2, principal point cx cy,
    aabb_scale 4 -> 3 cascades and cone stepping) through generate_training_samples_nerf's
    uv_to_ray(..., lens) (testbed_nerf.cu:890-905; the Newton undistortion, common_device.cuh:294-330):
    bit-exact per ray (rays, sample counts, NerfCoordinates) for the OpenCV lens;
  * the same with the fisheye model: atan differs by ulps between OCML and glibc, so ray directions are
    compared to 2e-6 relative and the sample counts to >= 99 % of the rays;
  * the NeRF camera rays of a frame with render_with_lens_distortion (testbed_nerf.cu:2504) for the OpenCV,
    fisheye, LatLong and Equirectangular lenses on the lego snapshot: the frame against the oracle's
    (PSNR >= 40 dB, >= 99.5 % of pixels within 2/255), and different from the Perspective frame.
"""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.oracle_mode("literal")]   # the oracle compares the reference's text as written

torch = pytest.importorskip("torch")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FOX = os.path.join(REPO, "data", "nerf", "fox270")
BATCH = 1 << 14
FISHEYE = (4, [0.05, -0.02, 0.004, -0.001, 0, 0, 0])


@pytest.fixture(scope="module")
def fox():
    from synerfgine_amd import Engine, Testbed, nerf_data, synthetic
    d = nerf_data.load_nerf(FOX, max_images=6)
    assert d["aabb_scale"] == 4 and all(l[0] == nerf_data.LENS_OPENCV for l in d["lenses"])
    tb = Testbed(0)
    cfg, params = synthetic.random_init(1337, aabb_scale=d["aabb_scale"])
    tb.set_nerf_model(cfg, params)
    eng = Engine(tb)
    eng.set_param("train_batch", BATCH)
    tb.set_training_dataset(d["images"], d["xforms"], d["focal"], d["pp"])
    tb.set_training_lens(d["lenses"])
    tb.train_reset(1337)
    st = tb.train(64)
    yield dict(tb=tb, eng=eng, cfg=cfg, d=d, stats=st)
    tb.close()


def _generate(T):
    """stage 1 of the next training step on the GPU, and the oracle's samples of the same batch"""
    import oracle as O
    import train_ref as R
    tb = T["tb"]
    ctrl = tb.train_debug(1, "ctrl", np.uint32)[:4].copy()
    nr = int(ctrl[0])
    g = dict(ctrl=ctrl, n_rays=int(T["stats"]["rays_per_batch"]), step=int(T["stats"]["step"]))
    g["ray_indices"] = tb.train_debug(0, "ray_indices", np.uint32)[:nr].copy()
    g["numsteps"] = tb.train_debug(0, "numsteps", np.uint32)[: 2 * nr].reshape(nr, 2).copy()
    g["rays"] = tb.train_debug(0, "rays", np.float32)[: 8 * nr].reshape(nr, 8).copy()
    g["coords"] = tb.train_debug(0, "coords", np.float32)[: 7 * int(ctrl[1])].reshape(-1, 7).copy()
    d = T["d"]
    vol = O.make_volume(tb.density_grid_bitfield(), aabb_scale=d["aabb_scale"])
    rng = R.step_rng(1337, g["step"])
    ns, rays, co = O.train_generate(vol, d["images"], d["xforms"], d["focal"], d["pp"], rng.state, rng.inc, g["n_rays"], max_per_ray=1024)
    return g, ns, rays, co


@pytest.mark.parametrize("lanes", [8, 1, 16], ids=["8_lanes", "one_lane", "16_lanes"])
def test_fox_opencv_train_generate_matches_oracle(fox, lanes):
    """The cascaded (aabb_scale 4, cone-stepped) generator in each form (train_gen_lanes) against the oracle, bit-exact."""
    fox["eng"].set_param("train_gen_lanes", lanes)
    try:
        _check_fox_opencv(fox)
    finally:
        fox["eng"].set_param("train_gen_lanes", 8)


def _check_fox_opencv(fox):
    import oracle as O
    O.set_train_lens(fox["d"]["lenses"])
    g, ns, rays, co = _generate(fox)
    nr = int(g["ctrl"][0])
    assert nr > 32, "too few training rays hit the occupancy grid"
    assert int(g["ctrl"][1]) == int(ns.sum())
    mb = int(fox["stats"]["measured_batch_before_compaction"])
    max_samples = 16 * BATCH if mb == 0 else (min(mb, 16 * BATCH) + 255) // 256 * 256   # train_nerf_step max_samples
    # every ray the oracle finds samples on is on the GPU list, and nothing else -- unless the sample budget overflowed:
    # the dropped rays then depend on the order of the reservations (atomics in the reference too)
    got = set(g["ray_indices"].tolist())
    if int(g["ctrl"][1]) <= max_samples:
        assert sorted(got) == np.nonzero(ns)[0].tolist()
    else:
        assert got <= set(np.nonzero(ns)[0].tolist())
    for k in range(nr):
        i = int(g["ray_indices"][k])
        n, base = g["numsteps"][k]
        assert n == ns[i], f"ray {i}: {n} samples on the GPU, {ns[i]} in the oracle"
        np.testing.assert_array_equal(g["rays"][k, [0, 1, 2, 4, 5, 6]], rays[i], err_msg=f"ray {i} origin/direction")
        m = min(int(n), 1024)
        assert np.array_equal(g["coords"][base:base + m].view(np.uint32), co[i, :m].view(np.uint32)), f"ray {i}: NerfCoordinates differ"
    # the lens moved the rays: a Perspective oracle disagrees
    O.set_train_lens([])
    _, ns_p, rays_p, _ = _generate(fox)
    moved = np.abs(rays_p[:, 3:] - rays[:, 3:]).max(axis=1) > 1e-4
    assert moved.mean() > 0.5


def test_fox_fisheye_train_generate_close_to_oracle(fox):
    import oracle as O
    tb = fox["tb"]
    n = len(fox["d"]["lenses"])
    tb.set_training_lens([FISHEYE] * n)
    O.set_train_lens([FISHEYE] * n)
    try:
        g, ns, rays, co = _generate(fox)
        nr = int(g["ctrl"][0])
        assert nr > 32
        idx = g["ray_indices"].astype(np.int64)
        gd, od = g["rays"][:, 4:7], rays[idx, 3:6]
        assert np.abs(gd - od).max() <= 2e-6 * np.abs(od).max(), "fisheye ray directions beyond 2e-6 relative"
        same = (g["numsteps"][:, 0] == ns[idx]).mean()   # (the GPU's rays only: the sample budget may drop some)
        assert same >= 0.99, f"{same:.4f} of the rays have the oracle's sample count"
    finally:
        tb.set_training_lens(fox["d"]["lenses"])


def _psnr(a, b):
    mse = float(np.mean((np.clip(a, 0, 1) - np.clip(b, 0, 1)) ** 2))
    return 10 * np.log10(1.0 / max(mse, 1e-12))


@pytest.mark.parametrize("lens", [(1, [0.0578421, -0.0805099, -0.000980296, 0.00015575]), FISHEYE, (3, []), (5, [])],
                         ids=["opencv", "fisheye", "latlong", "equirectangular"])
def test_render_lens_frame_matches_oracle(lens):
    import oracle as O
    from synerfgine_amd import scene as S
    if not os.path.exists(S.LEGO_INGP):
        pytest.skip("data/lego.ingp not present")
    tb, eng, (cfg, params, grid) = S.make_engine("c2", width=200, height=160, model="lego")
    try:
        tb.set_camera_view((0.62, -0.46, -0.64), (0.5, 0.5, 0.5), 1.2)
        persp = eng.frame(spp=0, reset=True).download("final_rgba")
        tb.set_render_lens(*lens)
        assert tb.render_lens()[0] == lens[0]
        eng.set_param("render_with_lens_distortion", 1)
        nrng, mrng = eng.rng_states(0).copy(), eng.rng_states(1).copy()
        got = eng.frame(spp=0, reset=True).download("final_rgba")
        O.set_render_lens(*lens)
        ref = O.render_frame(O.Model(cfg, params), O.volume_for(cfg, grid), tb, eng, nrng, mrng)["final"]
        assert np.isfinite(got).all()
        p = _psnr(got[..., :3], ref[..., :3])
        c = float((np.abs(np.clip(got, 0, 1) - np.clip(ref, 0, 1))[..., :3].max(axis=-1) <= 2 / 255).mean())
        assert p >= 40.0 and c >= 0.995, f"PSNR {p:.2f} dB, {c:.4f} of pixels within 2/255"
        assert _psnr(got[..., :3], persp[..., :3]) < 35.0, "the lens did not change the frame"
    finally:
        tb.close()


@pytest.mark.parametrize("where", ["global", "metadata"])
def test_snapshot_legacy_camera_distortion_key(tmp_path, where, synthetic_model):
    """from_json(NerfDataset) (json_binding.h:141-160) also accepts the legacy key "camera_distortion", at the dataset's
    global level and per image, and it overrides "lens": load_snapshot's render lens follows it."""
    import zlib

    import msgpack
    from synerfgine_amd import Testbed, ingp
    cfg, params, grid = synthetic_model
    p = tmp_path / "legacy.ingp"
    ingp.write_ingp(str(p), cfg, params, grid)
    root = msgpack.unpackb(zlib.decompress(p.read_bytes()), raw=False, strict_map_key=False)
    ds = root["snapshot"]["nerf"]["dataset"]
    lens = {"k1": 0.125, "k2": -0.0625, "p1": 0.001, "p2": 0.002}
    if where == "global":
        ds["lens"] = {}
        ds["camera_distortion"] = lens
    else:
        ds["metadata"] = [{"lens": {}, "camera_distortion": lens}]
    p.write_bytes(zlib.compress(msgpack.packb(root, use_bin_type=True), 6))
    tb = Testbed(0)
    try:
        tb.load_snapshot(str(p))
        mode, prm = tb.render_lens()
    finally:
        tb.close()
    assert mode == 1   # ELensMode::OpenCV
    np.testing.assert_allclose(prm[:4], [0.125, -0.0625, 0.001, 0.002], rtol=0, atol=1e-7)
