"""CPU tests of the lens models and the real-capture dataset loader (no GPU):

  * synerfgine_amd.nerf_data.load_nerf on the reference's fox capture (data/nerf/fox270, tools/make_fox.py): the
    frames read_lens / read_focal_length / the sharpness branch keep (nerf_loader.cu:175-270, 364-386), the OpenCV
    lens, principal point and focal length, aabb_scale 4;
  * the oracle's uv_to_ray undistortion (common_device.cuh:294-330, 403-447): the Newton iterate solves
    x + delta(x) = x0 -- the forward distortion pos_to_uv applies (507-541) maps it back to the pixel -- for the fox
    OpenCV lens and a fisheye lens, against a float64 restatement of the same Newton;
  * LatLong / Equirectangular directions are unit vectors with the documented axes; F-Theta's invalid domain.
"""
import json
import math
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FOX = os.path.join(REPO, "data", "nerf", "fox270")
FOX_LENS = (1, [0.0578421, -0.0805099, -0.000980296, 0.00015575])
FISHEYE = (4, [0.05, -0.02, 0.004, -0.001])


def test_fox_loader_reads_the_lens_and_keeps_frames_with_images():
    from synerfgine_amd import nerf_data as N
    meta = json.load(open(os.path.join(FOX, "transforms.json")))
    have = [f for f in meta["frames"] if os.path.exists(os.path.join(FOX, f["file_path"]))]
    assert len(meta["frames"]) == 67 and len(have) == 50
    d = N.load_nerf(FOX)
    assert d["images"].shape == (50, 480, 270, 4)
    assert d["paths"] == [f["file_path"] for f in have]
    assert d["aabb_scale"] == 4 and d["scale"] == N.NERF_SCALE and d["offset"] == (0.5, 0.5, 0.5)
    for mode, params in d["lenses"]:
        assert mode == N.LENS_OPENCV
        np.testing.assert_array_equal(np.float32(params[:4]), np.float32([meta["k1"], meta["k2"], meta["p1"], meta["p2"]]))
    np.testing.assert_array_equal(d["pp"][0], np.float32([np.float32(meta["cx"]) / np.float32(meta["w"]), np.float32(meta["cy"]) / np.float32(meta["h"])]))
    np.testing.assert_allclose(d["focal"][0], [meta["fl_x"], meta["fl_y"]], rtol=1e-6)
    # nerf_matrix_to_ngp of the first kept frame
    np.testing.assert_allclose(d["xforms"][0], N.nerf_matrix_to_ngp(have[0]["transform_matrix"]), rtol=0, atol=0)


def test_read_lens_rules():
    from synerfgine_amd import nerf_data as N
    lens, pp, rs = [0, [0.0] * 7], [0.5, 0.5], [0.0] * 4
    N.read_lens({"k1": 0.0, "k2": 0.0}, lens, pp, rs)
    assert lens[0] == N.LENS_PERSPECTIVE                       # all-zero coefficients stay Perspective
    N.read_lens({"k1": 0.1, "is_fisheye": True, "k3": 0.2, "k4": 0.3}, lens, pp, rs)
    assert lens[0] == N.LENS_OPENCV_FISHEYE and lens[1][2] == np.float32(0.2)
    N.read_lens({"cx": 10.0, "w": 40.0}, lens, pp, rs)
    assert lens[0] == N.LENS_OPENCV_FISHEYE and pp[0] == 0.25  # an outer mode is not overridden by nothing
    N.read_lens({"latlong": True}, lens, pp, rs)
    assert lens[0] == N.LENS_LATLONG
    fo = [0.0, 0.0]
    assert N.read_focal_length({"camera_angle_x": 0.5}, fo, (100, 50)) and fo[0] == fo[1] == pytest.approx(50 / math.tan(0.25))
    assert N.read_focal_length({"fl_x": 7.0, "camera_angle_x": 0.5, "y_fov": 90.0}, fo, (100, 50)) and fo == [7.0, pytest.approx(25.0)]


def _delta64(lens, u, v):
    mode, p = lens
    if mode == 4:
        r = math.hypot(u, v)
        if r <= 2.22e-16:
            return 0.0, 0.0
        th = math.atan(r)
        thd = th * (1 + p[0] * th ** 2 + p[1] * th ** 4 + p[2] * th ** 6 + p[3] * th ** 8)
        return u * thd / r - u, v * thd / r - v
    k1, k2, p1, p2 = p[:4]
    r2 = u * u + v * v
    rad = k1 * r2 + k2 * r2 * r2
    return u * rad + 2 * p1 * u * v + p2 * (r2 + 2 * u * u), v * rad + 2 * p2 * u * v + p1 * (r2 + 2 * v * v)


def _undistort64(lens, x0u, x0v):
    xu, xv = x0u, x0v
    for _ in range(100):
        du, dv = _delta64(lens, xu, xv)
        h = 1e-7
        a = _delta64(lens, xu + h, xv)
        b = _delta64(lens, xu, xv + h)
        j = np.array([[1 + (a[0] - du) / h, (b[0] - du) / h], [(a[1] - dv) / h, 1 + (b[1] - dv) / h]])
        s = np.linalg.solve(j, [xu + du - x0u, xv + dv - x0v])
        xu, xv = xu - s[0], xv - s[1]
        if s @ s < 1e-24:
            break
    return xu, xv


@pytest.mark.parametrize("lens", [FOX_LENS, FISHEYE], ids=["opencv", "fisheye"])
def test_oracle_undistortion_inverts_the_distortion(oracle_lib, lens):
    O = oracle_lib
    rng = np.random.default_rng(5)
    W, H, focal, sc = 270, 480, (343.88, 343.6225), (0.5134796, 0.5027438)
    worst_fwd, worst_ref = 0.0, 0.0
    for uv in rng.uniform(0.0, 1.0, size=(400, 2)).astype(np.float32):
        ok, d = O.uv_to_ray_dir(lens, uv, (W, H), focal, sc)
        assert ok and d[2] == 1.0
        x0 = ((np.float32(uv[0]) - np.float32(sc[0])) * np.float32(W) / np.float32(focal[0]),
              (np.float32(uv[1]) - np.float32(sc[1])) * np.float32(H) / np.float32(focal[1]))
        du, dv = O.lens_distortion_delta(lens, d[0], d[1])
        worst_fwd = max(worst_fwd, abs(d[0] + du - x0[0]), abs(d[1] + dv - x0[1]))
        ru, rv = _undistort64(lens, float(x0[0]), float(x0[1]))
        worst_ref = max(worst_ref, abs(d[0] - ru), abs(d[1] - rv))
    assert worst_fwd < 2e-6, worst_fwd   # pos_to_uv of the undistorted direction lands on the pixel
    assert worst_ref < 2e-6, worst_ref   # and it is the float64 Newton's solution


def test_oracle_latlong_equirect_ftheta_directions(oracle_lib):
    O = oracle_lib
    ok, d = O.uv_to_ray_dir((3, []), (0.5, 0.5), (64, 32), (1, 1), (0.5, 0.5))
    assert ok and np.allclose(d, [0, 0, 1])
    ok, d = O.uv_to_ray_dir((3, []), (0.75, 0.5), (64, 32), (1, 1), (0.5, 0.5))
    assert ok and np.allclose(d, [1, 0, 0], atol=1e-6)
    ok, d = O.uv_to_ray_dir((5, []), (0.5, 1.0), (64, 32), (1, 1), (0.5, 0.5))
    assert ok and np.allclose(d, [0, 1, 0], atol=1e-6)
    for uv in np.random.default_rng(1).uniform(0, 1, size=(50, 2)):
        for mode in (3, 5):
            ok, d = O.uv_to_ray_dir((mode, []), uv, (64, 32), (1, 1), (0.5, 0.5))
            assert ok and abs(np.linalg.norm(d) - 1.0) < 1e-5
    # F-Theta: angle polynomial in the pixel radius; the principal point (norm 0) is invalid
    ft = (2, [0.0, 1e-3, 0.0, 0.0, 0.0, 640.0, 480.0])
    ok, _ = O.uv_to_ray_dir(ft, (0.5, 0.5), (640, 480), (1, 1), (0.5, 0.5))
    assert not ok
    ok, d = O.uv_to_ray_dir(ft, (0.6, 0.5), (640, 480), (1, 1), (0.5, 0.5))
    assert ok and d[1] == 0.0 and np.isclose(math.atan2(d[0], d[2]), 1e-3 * 64.0, rtol=1e-5)


def test_loader_sorts_frames_naturally_before_the_cull(tmp_path):
    """load_nerf sorts the frames by file_path in natural order (SI::natural::compare, nerf_loader.cu:347-349) before
    the n_frames cull, and converts fields of view with the float expressions of fov_to_focal_length
    (common_device.cuh:618-620)."""
    from synerfgine_amd import nerf_data
    img = np.zeros((4, 6, 4), np.uint8)
    names = ["r_10", "r_2", "r_1", "r_1a"]
    for k, n in enumerate(names):
        img[..., 0] = k
        _write_png(tmp_path / f"{n}.png", img)
    eye = [[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]]
    meta = {"camera_angle_x": 0.6911112070083618, "n_frames": 3,
            "frames": [{"file_path": f"./{n}.png", "transform_matrix": eye} for n in names]}
    (tmp_path / "transforms.json").write_text(json.dumps(meta))
    d = nerf_data.load_nerf(str(tmp_path))
    assert d["paths"] == ["./r_1.png", "./r_1a.png", "./r_2.png"]   # natural order, then the first n_frames
    assert [int(x[0, 0, 0]) for x in d["images"]] == [2, 3, 1]
    f32 = np.float32
    deg = f32(f32(f32(0.6911112070083618) * f32(180)) / f32(math.pi))
    ref = f32(f32(0.5) * f32(6)) / f32(np.tan(f32(f32(f32(0.5) * deg) * f32(math.pi)) / f32(180)))
    assert abs(d["focal"][0][0] - ref) <= 4e-7 * ref


def _write_png(path, img):
    import struct
    import zlib
    h, w = img.shape[:2]
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))
    def chunk(t, data):
        return struct.pack(">I", len(data)) + t + data + struct.pack(">I", zlib.crc32(t + data) & 0xFFFFFFFF)
    path.write_bytes(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)) + chunk(b"IDAT", zlib.compress(raw)) +
                     chunk(b"IEND", b""))
