"""Headless display stage: the oracle's restatement of main.frag's FXAA
(scripts/virtual_desc/main.frag:50-97) and the blend/readback of Display::present / save_image
(display.cu:265-322) -- known answers on CPU -- and the PNG writer round trip."""
import numpy as np
import pytest


def test_fxaa_flat_image_is_identity(oracle_lib):
    img = np.zeros((16, 20, 4), np.float32)
    img[..., :3] = [0.2, 0.4, 0.6]
    img[..., 3] = 1.0
    out = oracle_lib.display(img)
    assert (out == np.round(np.array([0.2, 0.4, 0.6]) * 255).astype(np.uint8)).all()


def test_fxaa_blend_over_clear_colour(oracle_lib):
    img = np.zeros((8, 8, 4), np.float32)   # transparent black: the clear colour shows
    out = oracle_lib.display(img, clear=(1.0, 0.0, 0.5))
    assert (out == [255, 0, 128]).all()


def test_fxaa_smooths_a_diagonal_edge_only_there(oracle_lib):
    """FXAA blends along the local edge direction: an axis-aligned edge stays sharp, a staircase
    (diagonal) edge gets intermediate values, flat regions away from it are untouched."""
    img = np.zeros((32, 32, 4), np.float32)
    img[..., 3] = 1.0
    img[:, 16:, :3] = 1.0
    out = oracle_lib.display(img).astype(np.int32)
    assert ((out == 0) | (out == 255)).all()
    yy, xx = np.mgrid[0:32, 0:32]
    img[..., :3] = ((xx + 0.5 * yy) > 20)[..., None].astype(np.float32)
    out = oracle_lib.display(img).astype(np.int32)
    d = np.abs((xx + 0.5 * yy) - 20)
    far = (d > 4) & (xx > 1) & (xx < 30) & (yy > 1) & (yy < 30)
    assert (out[far, 0] == np.where((xx + 0.5 * yy)[far] > 20, 255, 0)).all()
    near = out[d <= 1.5, 0]
    assert ((near > 0) & (near < 255)).any()


def test_fxaa_window_resampling_and_wrap(oracle_lib):
    rng = np.random.default_rng(0)
    img = rng.uniform(0, 1, (12, 10, 4)).astype(np.float32)
    img[..., 3] = 1.0
    out = oracle_lib.display(img, out_w=20, out_h=24)
    assert out.shape == (24, 20, 3)


def test_png_writer_round_trip(tmp_path):
    from synerfgine_amd import nerf_data, write_png
    rng = np.random.default_rng(1)
    for ch in (3, 4):
        im = rng.integers(0, 256, (17, 23, ch), dtype=np.uint8)
        p = tmp_path / f"im{ch}.png"
        write_png(p, im)
        back = nerf_data.read_png(p)
        assert np.array_equal(back[..., :ch], im)
        if ch == 3:
            assert (back[..., 3] == 255).all()
