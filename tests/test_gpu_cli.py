"""sng-render on the GPU: the profiling.sh-style command line renders frames and writes PNGs; the written
frame is the final image the library renders for the same inputs through the Python host mirror
(sng_final_rgba8), byte for byte."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "synerfgine_amd", "_build", "sng-render")


def test_cli_renders_the_library_frame(tmp_path):
    if not os.path.exists(CLI):
        pytest.fail("sng-render not built (make -C synerfgine_amd)")
    out = tmp_path / "frames"
    W, H = 320, 180
    r = subprocess.run([CLI, "--snapshot", os.path.join(REPO, "data", "lego.ingp"), "--virtual", os.path.join(REPO, "scenes", "armadillo.json"),
                        "--frag", "main.frag", "--width", str(W), "--height", str(H), "--sshadows", "2", "--nshadows", "1", "--frames", "2",
                        "--out", str(out)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("frame=")]
    assert len(lines) == 2 and '"frames_per_s"' in r.stdout
    files = sorted(os.listdir(out))
    assert files == ["frame-0000.png", "frame-0001.png"]

    from synerfgine_amd import Engine, Testbed
    from synerfgine_amd.nerf_data import read_png
    img = read_png(str(out / "frame-0001.png"))
    tb = Testbed(0)
    try:
        tb.load_snapshot(os.path.join(REPO, "data", "lego.ingp"))
        eng = Engine(tb)
        eng.set_virtual_world(os.path.join(REPO, "scenes", "armadillo.json"))
        eng.init(W, H)
        eng.set_param("sshadows", 2)
        eng.set_param("nshadows", 1)
        eng.frame(spp=0, reset=True)
        f = eng.frame(spp=0, reset=True).download("final_rgba").astype(np.float32).reshape(H, W, 4)
        # sng_final_rgba8's encoding (display.hip rgba8_band_kernel): (int)(clamp(c, 0, 1) * 255 + 0.5)
        c = np.fmin(np.fmax(f, np.float32(0)), np.float32(1))
        ref = (c * np.float32(255) + np.float32(0.5)).astype(np.int32).astype(np.uint8)
    finally:
        tb.close()
    assert img.shape == (H, W, 4)
    assert np.array_equal(img, ref)
