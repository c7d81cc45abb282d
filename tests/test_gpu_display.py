"""GPU: the headless display stage (display.hip; main.frag FXAA + blend + RGB8 readback,
display.cu:265-322) against the oracle's restatement on the same final frame (bit-exact), and
Display::save_image's numbering / image budget."""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.oracle_mode("literal")]   # the oracle compares the reference's text as written
torch = pytest.importorskip("torch")


def test_display_matches_oracle_and_records(tmp_path, oracle_lib):
    from synerfgine_amd import nerf_data
    from synerfgine_amd import scene as S
    tb, eng, _ = S.make_engine("c3", width=160, height=90, overrides={"res_factor": 8})
    r = eng.frame()
    final = r.download("final_rgba").copy()
    got = eng.display()
    exp = oracle_lib.display(final)
    diff = np.abs(got.astype(np.int32) - exp.astype(np.int32))
    assert diff.max() <= 1 and (diff == 0).mean() >= 0.999, (int(diff.max()), float((diff == 0).mean()))
    eng.set_param("img_count_max", 2)
    written = [eng.save_image(tmp_path) for _ in range(4)]
    tb.close()
    assert written == [True, True, True, False]   # save_image refuses once count > img_count_max
    names = sorted(os.listdir(tmp_path))
    assert names == ["output-001.png", "output-002.png", "output-003.png"]
    back = nerf_data.read_png(tmp_path / "output-001.png")
    assert np.array_equal(back[..., :3], got)
