"""NeRF soft shadows with a neighbourhood (nerf_shadow_samples > 0, kernel r = 2): the reference's
shadow_for_px draws each neighbour's light sample from the NEIGHBOUR's XORWOW state, rand_state[idx]
with idx the neighbour's pixel (testbed_nerf.cu:1635,1649, called from shade_with_shadow 1769-1772) --
many threads advance one state at once, a data race with no defined result. This library draws a
pixel's whole neighbourhood from the pixel's own stream (DESIGN.md decision 10): deterministic, and the
same draws for r = 0.

The two can only agree in distribution. The oracle runs both: its default (the GPU kernels' semantics,
checked against the GPU in tests/test_gpu_parity.py) and `orc_set_shadow_rng_mode(1)`, the reference's
sharing with the pixels serialised in index order (one race-free interleaving). Over K independent
seeds the per-pixel mean shadow factor of the two must agree within the statistical error, on a
penumbra of an area light behind a square occluder (no NeRF occupancy: the mesh term alone).
CPU only: the oracle is the checker here, nothing is measured.
"""
import ctypes

import numpy as np

W, H, K, R = 24, 24, 48, 2


def _scene(O):
    # occluder: a 0.3 x 0.3 square (two triangles) at z = 0.5 above the receiver plane z = 0
    a, b = 0.35, 0.65
    tris = np.array([[[a, a, 0.5], [b, a, 0.5], [b, b, 0.5]], [[a, a, 0.5], [b, b, 0.5], [a, b, 0.5]]], np.float32)
    cap = 16
    nodes = np.zeros((cap, 8), np.float32)
    n = O.lib().orc_bvh_build(O.ptr(tris), len(tris), 4, O.ptr(nodes), cap)
    obj = dict(nodes=nodes[:n].copy(), tris=tris, rot=np.eye(3, dtype=np.float32).ravel(order="F"), pos=np.zeros(3, np.float32),
               scale=1.0, mat_id=0)
    objs = O.make_objects([obj])
    lights = O.make_lights([{"pos": [0.35, 0.35, 1.0], "intensity": 1.0, "size": 0.3, "type": 0}])
    u = (np.arange(W, dtype=np.float32) + 0.5) / W
    v = (np.arange(H, dtype=np.float32) + 0.5) / H
    pos = np.zeros((H, W, 3), np.float32)
    pos[..., 0], pos[..., 1] = np.meshgrid(u, v)
    nrm = np.zeros((H, W, 3), np.float32)
    nrm[..., 2] = 1.0
    vol = O.make_volume(np.zeros(128 ** 3 // 8 * 8, np.uint8))   # empty occupancy: the NeRF term is 1
    return objs, lights, pos, nrm, vol


def _shadow(O, objs, lights, pos, nrm, vol, seed, neighbour):
    rng = O.xorwow_states(W * H, seed=seed)
    rgba = np.ones((H, W, 4), np.float32)   # srgb_to_linear(1) = 1: the output is the shadow factor
    res = np.array([W, H], np.int32)
    O.lib().orc_set_shadow_rng_mode(1 if neighbour else 0)
    try:
        O.lib().orc_shade_nerf_shadows(ctypes.byref(vol), O.ptr(res), O.ptr(rgba), O.ptr(pos), O.ptr(nrm), objs, 1, lights, 1, O.ptr(rng),
                                       1.0, 0.0, 2 * R + 1)
    finally:
        O.lib().orc_set_shadow_rng_mode(0)
    return rgba[..., 0].copy()


def test_neighbour_rng_sharing_matches_in_distribution(oracle_lib):
    O = oracle_lib
    objs, lights, pos, nrm, vol = _scene(O)
    own = np.stack([_shadow(O, objs, lights, pos, nrm, vol, 1000 + k, False) for k in range(K)])
    shared = np.stack([_shadow(O, objs, lights, pos, nrm, vol, 1000 + k, True) for k in range(K)])
    pen = (own.std(axis=0) > 1e-3) | (shared.std(axis=0) > 1e-3)   # the penumbra: pixels whose value is random
    assert pen.mean() > 0.1, "the scene must have a penumbra"
    assert not np.array_equal(own, shared)   # different draws per trial...
    d = own.mean(axis=0) - shared.mean(axis=0)
    se = np.sqrt((own.var(axis=0, ddof=1) + shared.var(axis=0, ddof=1)) / K) + 1e-6
    z = np.abs(d[pen]) / se[pen]
    # ...the same expected shadow per pixel: |z| < 4.5 on every penumbra pixel, and the frame mean within 0.5 %
    assert z.max() < 4.5, f"max |z| {z.max():.2f} over {pen.sum()} penumbra pixels"
    assert abs(own.mean() - shared.mean()) < 5e-3 * own.mean()
    # and the same spread per trial (the neighbourhood average of 25 independent light samples either way)
    ratio = own.std(axis=0)[pen].mean() / shared.std(axis=0)[pen].mean()
    assert 0.8 < ratio < 1.25, ratio


def test_rng_modes_agree_without_neighbourhood(oracle_lib):
    """r = 0 (the reference default, nerf_shadow_samples 0): the centre pixel IS the neighbour, bit-identical."""
    O = oracle_lib
    objs, lights, pos, nrm, vol = _scene(O)
    outs = []
    for neighbour in (False, True):
        rng = O.xorwow_states(W * H, seed=7)
        rgba = np.ones((H, W, 4), np.float32)
        res = np.array([W, H], np.int32)
        O.lib().orc_set_shadow_rng_mode(1 if neighbour else 0)
        try:
            O.lib().orc_shade_nerf_shadows(ctypes.byref(vol), O.ptr(res), O.ptr(rgba), O.ptr(pos), O.ptr(nrm), objs, 1, lights, 1, O.ptr(rng), 1.0, 0.0, 1)
        finally:
            O.lib().orc_set_shadow_rng_mode(0)
        outs.append((rgba, rng))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
