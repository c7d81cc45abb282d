"""The raytracer's ImgBufferType views (RayTracer::m_buffer_to_show, raytracer.cuh:20-30,179; written by sng::raytrace
at raytracer.cu:189-216): Next/Src Origin, Next/Src Direction, Normal, Depth and NerfShadow, selected by the
rt_buffer_type parameter, against the oracle's raytrace of the same inputs.  The views come from the one-kernel path
(the deferred shadow queues carry only the Final colour); the NeRF layer is hidden so the frame is the view itself.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VIEWS = {1: "next_origin", 2: "src_origin", 3: "next_direction", 4: "src_direction", 5: "normal", 6: "depth", 7: "nerf_shadow"}


def _psnr(a, b):
    mse = float(np.mean((np.clip(a, 0, 1) - np.clip(b, 0, 1)) ** 2))
    return 10 * np.log10(1.0 / max(mse, 1e-12))


@pytest.mark.parametrize("view", sorted(VIEWS), ids=[VIEWS[k] for k in sorted(VIEWS)])
def test_raytracer_buffer_view_matches_oracle(view):
    import oracle as O
    from synerfgine_amd import _lib
    from synerfgine_amd import scene as S
    tb, eng, (cfg, params, grid) = S.make_engine("c3", width=160, height=90,
                                                 overrides={"res_factor": 8, "show_nerf": 0, "srgb": 0, "rt_buffer_type": view})
    try:
        nrng, mrng = eng.rng_states(0).copy(), eng.rng_states(1).copy()
        fin = eng.frame(spp=0, reset=True).download("final_rgba")
        with O.literal(0):
            ref = O.render_frame(O.Model(cfg, params), O.volume_for(cfg, grid), tb, eng, nrng, mrng)["final"]
        eng.set_param("rt_buffer_type", 0)
        final_view = eng.frame(spp=0, reset=True).download("final_rgba")
        with pytest.raises(_lib.SngError):
            eng.set_param("rt_buffer_type", 8)
    finally:
        tb.close()
    hit = np.isfinite(ref[..., :3]).all(axis=-1)
    assert hit.mean() > 0.5
    # NaN where the reference normalises a zero sum (a miss has pos / normal 0): both sides, same pixels
    assert np.array_equal(np.isfinite(fin[..., :3]).all(axis=-1), hit)
    a, b = fin[hit][:, :3], ref[hit][:, :3]
    p = _psnr(a, b)
    close = float((np.abs(np.clip(a, 0, 1) - np.clip(b, 0, 1)).max(axis=-1) <= 2 / 255).mean())
    assert p >= 40.0 and close >= 0.995, f"{VIEWS[view]}: PSNR {p:.2f} dB, {close:.4f} within 2/255"
    # the view is not the Final colour
    assert not np.array_equal(np.nan_to_num(fin), np.nan_to_num(final_view))
