"""Known-answer tests that pin the CPU oracle's restated primitives (CPU only).

The reference ships no golden vectors and its tiny-cuda-nn / cuRAND dependencies are not
vendored, so each primitive is pinned against an INDEPENDENT source:
  * Morton codes          -- bit-interleaving definition (tcnn common_device.h);
  * Sobol directions      -- scipy.stats.qmc.Sobol (Joe-Kuo), re-indexed from Gray-code order;
  * XORWOW                -- Marsaglia's published xorwow recurrence + cuRAND's seeding constants
                             restated in pure Python; jump-ahead matrices vs stepping;
  * hash-grid level table -- SURVEY.md Appendix B (computed with the reference's float expressions);
  * SH degree 4           -- orthonormality of the real SH basis on the sphere;
  * fp16 conversion       -- numpy's IEEE binary16 round-to-nearest-even.
"""
import numpy as np
import pytest


def test_morton_known_answers(oracle_lib):
    L = oracle_lib.lib()
    assert L.orc_morton3D(0, 0, 0) == 0
    assert L.orc_morton3D(1, 0, 0) == 1 and L.orc_morton3D(0, 1, 0) == 2 and L.orc_morton3D(0, 0, 1) == 4
    assert L.orc_morton3D(127, 127, 127) == (1 << 21) - 1
    rng = np.random.default_rng(0)
    for x, y, z in rng.integers(0, 128, (200, 3)):
        code = 0
        for b in range(7):
            code |= ((int(x) >> b) & 1) << (3 * b) | ((int(y) >> b) & 1) << (3 * b + 1) | ((int(z) >> b) & 1) << (3 * b + 2)
        assert L.orc_morton3D(int(x), int(y), int(z)) == code
        assert L.orc_morton3D_invert(code) == x and L.orc_morton3D_invert(code >> 1) == y and L.orc_morton3D_invert(code >> 2) == z


def test_sobol_matches_scipy_joe_kuo(oracle_lib):
    qmc = pytest.importorskip("scipy.stats.qmc")
    L = oracle_lib.lib()
    n = 1024
    pts = qmc.Sobol(d=2, scramble=False).random(n)
    for k in range(n):
        g = k ^ (k >> 1)   # scipy walks the sequence in Gray-code order; random_val.cuh indexes it directly
        assert L.orc_sobol(g, 0) / 2.0 ** 32 == pts[k, 0]
        assert L.orc_sobol(g, 1) / 2.0 ** 32 == pts[k, 1]


def test_ld_random_pixel_offset_spp0_is_pixel_center_jitter(oracle_lib):
    import ctypes
    L = oracle_lib.lib()
    out = (ctypes.c_float * 2)()
    L.orc_ld_random_pixel_offset(0, out)
    assert 0.0 <= out[0] < 1.0 and 0.0 <= out[1] < 1.0
    vals = [L.orc_ld_random_val(i, 0x1234, 0) for i in range(256)]
    assert all(0.0 <= v < 1.0 for v in vals) and len(set(vals)) == 256


# ---- XORWOW: pure-Python restatement of the published generator --------------------------
M32 = 0xFFFFFFFF


def _py_xorwow_next(s):
    t = s[0] ^ (s[0] >> 2)
    s[0], s[1], s[2], s[3] = s[1], s[2], s[3], s[4]
    s[4] = (s[4] ^ ((s[4] << 4) & M32)) ^ (t ^ ((t << 1) & M32))
    s[5] = (s[5] + 362437) & M32
    return (s[5] + s[4]) & M32


def _py_curand_seed(seed):
    s0 = (seed & M32) ^ 0xAAD26B49
    s1 = (seed >> 32) ^ 0xF7DCEFDD
    t0 = (1099087573 * s0) & M32
    t1 = (2591861531 * s1) & M32
    return [(123456789 + t0) & M32, 362436069 ^ t0, (521288629 + t1) & M32, 88675123 ^ t1, (5783321 + t0) & M32,
            (6615241 + t1 + t0) & M32]


def _state(oracle_lib, seed, subseq=0, offset=0):
    st = np.zeros(6, np.uint32)
    oracle_lib.lib().orc_xorwow_init(seed, subseq, offset, oracle_lib.ptr(st))
    return st


@pytest.mark.parametrize("seed", [0, 1999, 0x123456789ABCDEF])
def test_xorwow_seeding_and_sequence(oracle_lib, seed):
    st = _state(oracle_lib, seed)
    py = _py_curand_seed(seed)
    assert st.tolist() == py
    L = oracle_lib.lib()
    for _ in range(1000):
        assert L.orc_xorwow_next(oracle_lib.ptr(st)) == _py_xorwow_next(py)
    # curand_uniform = x * 2^-32 + 2^-33  (in (0, 1])
    v = L.orc_curand_uniform(oracle_lib.ptr(st))
    x = _py_xorwow_next(py)
    assert v == np.float32(np.float32(x) * np.float32(2.0 ** -32) + np.float32(2.0 ** -33))


@pytest.mark.parametrize("k", [0, 1, 5, 13, 17])
def test_xorwow_jump_matrix_equals_stepping(oracle_lib, k):
    L = oracle_lib.lib()
    a = _state(oracle_lib, 77)
    b = a.copy()
    L.orc_xorwow_jump_matrix(oracle_lib.ptr(a), k)
    L.orc_xorwow_jump_steps_naive(oracle_lib.ptr(b), 1 << k)
    assert np.array_equal(a, b)


def test_xorwow_offset_and_subsequence(oracle_lib):
    L = oracle_lib.lib()
    # offset = plain skip-ahead in draws
    a = _state(oracle_lib, 1999, 0, 12345)
    b = _state(oracle_lib, 1999)
    L.orc_xorwow_jump_steps_naive(oracle_lib.ptr(b), 12345)
    assert np.array_equal(a, b)
    # subsequence i = jump of i * 2^67 draws: (i=3) == (i=1) + 2 jumps of 2^67
    c = _state(oracle_lib, 1999, 3)
    d = _state(oracle_lib, 1999, 1)
    L.orc_xorwow_jump_matrix(oracle_lib.ptr(d), 67)
    L.orc_xorwow_jump_matrix(oracle_lib.ptr(d), 67)
    assert np.array_equal(c, d)
    # the per-pixel init (init_rand_state: curand_init(PT_SEED, idx, 0)) equals the single-state init
    many = oracle_lib.xorwow_states(5)
    for i in range(5):
        assert np.array_equal(many[i], _state(oracle_lib, 1999, i))


# ---- hash-grid level table: SURVEY.md Appendix B --------------------------------------
APPENDIX_B = [
    # (L, F, per_level_scale float bits, resolutions, total entries)
    (8, 4, 0x40000000, [16, 32, 64, 128, 256, 512, 1024, 2048], 2920448),
    (8, 4, 0x403E350F, [16, 48, 142, 421, 1249, 3710, 11026, 32768], 3260416),
    (16, 2, 0x3FB0E285, [16, 23, 31, 43, 59, 81, 112, 154, 213, 295, 407, 562, 777, 1073, 1483, 2048], 6098120),
    (16, 2, 0x3FD4CC02, None, 6811592),
]


@pytest.mark.parametrize("L_,F,bits,res,entries", APPENDIX_B)
def test_level_table_matches_appendix_b(oracle_lib, L_, F, bits, res, entries):
    b = float(np.array([bits], np.uint32).view(np.float32)[0])
    cfg = dict(n_levels=L_, n_features_per_level=F, log2_hashmap_size=19, base_resolution=16, per_level_scale=b)
    offs, got_res = oracle_lib.level_table(cfg)
    if res is not None:
        assert got_res.tolist() == res
    assert int(offs[-1]) == entries
    m = oracle_lib.Model(cfg, np.zeros(1, np.float16))
    assert oracle_lib.lib().orc_n_params(m.ref()) == 3072 + 7168 + entries * F
    # dense levels are res^3 rounded to a multiple of 8, hashed ones are 2^19
    sizes = np.diff(offs.astype(np.int64))
    for r, s in zip(got_res, sizes):
        dense = (int(r) ** 3 + 7) // 8 * 8
        assert s == min(dense, 1 << 19)


def test_sh_basis_is_orthonormal(oracle_lib):
    # Fibonacci sphere quadrature; SH output of the oracle is fp16 so the tolerance is loose
    n = 20000
    i = np.arange(n) + 0.5
    phi = np.arccos(1 - 2 * i / n)
    th = np.pi * (1 + 5 ** 0.5) * i
    d = np.stack([np.cos(th) * np.sin(phi), np.sin(th) * np.sin(phi), np.cos(phi)], 1).astype(np.float32)
    coords = np.zeros((n, 7), np.float32)
    coords[:, 4:7] = (d + 1) * 0.5
    out = np.zeros((n, 16), np.uint16)
    oracle_lib.lib().orc_sh_encode(oracle_lib.ptr(coords), 7, 4, n, oracle_lib.ptr(out))
    Y = out.view(np.float16).astype(np.float64)
    G = Y.T @ Y * (4 * np.pi / n)
    assert np.allclose(G, np.eye(16), atol=2e-2), np.abs(G - np.eye(16)).max()
    assert abs(Y[0, 0] - 0.28209479177387814) < 1e-3


def test_fp16_conversion_matches_numpy(oracle_lib):
    L = oracle_lib.lib()
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.normal(0, 1, 3000), rng.normal(0, 1e-5, 500), rng.normal(0, 3e4, 500),
                         [0.0, -0.0, 65504.0, 65520.0, 1e-8, 6.1e-5, np.inf, -np.inf]]).astype(np.float32)
    with np.errstate(over="ignore"):
        ref = xs.astype(np.float16)
    for x, r in zip(xs, ref):
        h = L.orc_float_to_half(float(x))
        assert h == int(r.view(np.uint16)), x
        assert L.orc_half_to_float(h) == float(r)
