"""The oracle's hash-grid encoding and fused MLP against a vectorised numpy restatement (CPU only).

tiny-cuda-nn is not vendored in the reference, so its published algorithm
(GridEncoding with CoherentPrime hashing and fp16 FMA accumulation, SH degree 4,
FullyFusedMLP without bias) is restated twice, independently: in C++ (oracle/sng_oracle.cpp)
and here in numpy.  Encoding must agree bit for bit; the MLP (fp32 accumulation order differs:
numpy sums in float64) within 2 fp16 ulp + 1e-3.
"""
import numpy as np
import pytest

PRIMES = (np.uint64(1), np.uint64(2654435761), np.uint64(805459861))


def _np_level_params(cfg):
    L, Nmin = cfg["n_levels"], cfg["base_resolution"]
    log2b = np.float32(np.log2(np.float32(cfg["per_level_scale"])))
    out, off = [], 0
    for l in range(L):
        # grid_scale: exp2f(l * log2(b)) * Nmin - 1  (fma form); exact for b = 2
        scale = np.float32(np.float64(np.exp2(np.float32(l) * log2b)) * Nmin - 1.0)
        res = int(np.ceil(scale)) + 1
        size = min((res ** 3 + 7) // 8 * 8, 1 << cfg["log2_hashmap_size"])
        out.append((off, size, scale, res))
        off += size
    return out


def _np_encode(cfg, params, x):
    F = cfg["n_features_per_level"]
    grid_all = params[3072 + 7168:]
    n = x.shape[0]
    enc = np.zeros((n, cfg["n_levels"] * F), np.float16)
    for l, (off, size, scale, res) in enumerate(_np_level_params(cfg)):
        p = (np.float64(scale) * x.astype(np.float64) + 0.5).astype(np.float32)   # fmaf(scale, x, 0.5)
        fl = np.floor(p)
        pg = fl.astype(np.int64)
        w = (p - fl).astype(np.float32)
        acc = np.zeros((n, F), np.float16)
        dense = res ** 3 <= size
        for idx in range(8):
            weight = np.ones(n, np.float32)
            pl = []
            for d in range(3):
                if idx & (1 << d):
                    weight = (weight * w[:, d]).astype(np.float32)
                    pl.append(pg[:, d] + 1)
                else:
                    weight = (weight * (np.float32(1.0) - w[:, d])).astype(np.float32)
                    pl.append(pg[:, d])
            pl = [q.astype(np.uint64) for q in pl]
            if dense:
                index = (pl[0] + pl[1] * np.uint64(res) + pl[2] * np.uint64(res * res)) & np.uint64(0xFFFFFFFF)
            else:
                index = ((pl[0] * PRIMES[0]) ^ (pl[1] * PRIMES[1]) ^ (pl[2] * PRIMES[2])) & np.uint64(0xFFFFFFFF)
            index = (index % np.uint64(size)).astype(np.int64)
            vals = grid_all[off * F + index[:, None] * F + np.arange(F)[None, :]].astype(np.float64)
            wh = weight.astype(np.float16).astype(np.float64)
            acc = (wh[:, None] * vals + acc.astype(np.float64)).astype(np.float16)   # half fma, single rounding
        enc[:, l * F:(l + 1) * F] = acc
    return enc


def _np_sh(d):
    x, y, z = (d[:, 0] * 2 - 1), (d[:, 1] * 2 - 1), (d[:, 2] * 2 - 1)
    x, y, z = [v.astype(np.float64) for v in (x, y, z)]
    xy, xz, yz, x2, y2, z2 = x * y, x * z, y * z, x * x, y * y, z * z
    o = [np.full_like(x, 0.28209479177387814), -0.48860251190291987 * y, 0.48860251190291987 * z, -0.48860251190291987 * x,
         1.0925484305920792 * xy, -1.0925484305920792 * yz, 0.94617469575755997 * z2 - 0.31539156525251999,
         -1.0925484305920792 * xz, 0.54627421529603959 * (x2 - y2), 0.59004358992664352 * y * (-3 * x2 + y2),
         2.8906114426405538 * xy * z, 0.45704579946446572 * y * (1 - 5 * z2), 0.3731763325901154 * z * (5 * z2 - 3),
         0.45704579946446572 * x * (1 - 5 * z2), 1.4453057213202769 * z * (x2 - y2), 0.59004358992664352 * x * (-x2 + 3 * y2)]
    return np.stack(o, 1).astype(np.float16)


def _dense(W, n_out, n_in, h, relu):
    y = h.astype(np.float64) @ W.reshape(n_out, n_in).astype(np.float64).T
    if relu:
        y = np.maximum(y, 0)
    return y.astype(np.float16)


def _np_network(cfg, params, c):
    enc = _np_encode(cfg, params, c[:, :3])
    dW0, dW1 = params[0:2048], params[2048:3072]
    rW0, rW1, rW2 = params[3072:5120], params[5120:9216], params[9216:10240]
    h = _dense(dW0, 64, 32, enc, True)
    dens = _dense(dW1, 16, 64, h, False)
    rgb_in = np.concatenate([dens, _np_sh(c[:, 4:7])], 1)
    h = _dense(rW0, 64, 32, rgb_in, True)
    h = _dense(rW1, 64, 64, h, True)
    out = _dense(rW2, 16, 64, h, False)
    out[:, 3] = dens[:, 0]
    return out


def _coords(n, seed):
    rng = np.random.default_rng(seed)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = rng.uniform(0, 1, (n, 3))
    c[: n // 10, :3] = rng.integers(0, 2, (n // 10, 3))   # exact cube faces/corners: unclamped corner aliasing
    c[:, 3] = rng.uniform(0, 1, n)
    d = rng.normal(size=(n, 3))
    c[:, 4:7] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) * 0.5
    return c


@pytest.fixture(scope="module")
def small_model():
    """Base.json geometry with random weights large enough to make every level matter."""
    cfg = dict(n_levels=8, n_features_per_level=4, log2_hashmap_size=19, base_resolution=16, per_level_scale=2.0, aabb_scale=1)
    rng = np.random.default_rng(1337)
    import oracle as O
    n = O.lib().orc_n_params(O.Model(cfg, np.zeros(1, np.float16)).ref())
    p = np.empty(n, np.float16)
    p[:10240] = rng.uniform(-0.25, 0.25, 10240)
    p[10240:] = rng.uniform(-1.0, 1.0, n - 10240)
    return cfg, p


def test_level_table_numpy(oracle_lib, small_model):
    cfg, _ = small_model
    offs, res = oracle_lib.level_table(cfg)
    lv = _np_level_params(cfg)
    assert [r for (_, _, _, r) in lv] == res.tolist()
    assert [o for (o, _, _, _) in lv] == offs[:-1].tolist()


def test_encode_bit_exact_vs_numpy(oracle_lib, small_model):
    cfg, p = small_model
    c = _coords(3000, 5)
    got = oracle_lib.encode(oracle_lib.Model(cfg, p), c, 7)
    exp = _np_encode(cfg, p, c[:, :3])
    bad = np.argwhere(got.view(np.uint16) != exp.view(np.uint16))
    assert len(bad) == 0, f"{len(bad)} mismatches, first {bad[:5].tolist()}"


def test_network_vs_numpy(oracle_lib, small_model):
    cfg, p = small_model
    c = _coords(2000, 6)
    got = oracle_lib.inference(oracle_lib.Model(cfg, p), c).astype(np.float32)
    exp = _np_network(cfg, p, c).astype(np.float32)
    ulp = np.exp2(np.floor(np.log2(np.maximum(np.abs(exp), 6.1e-5))) - 10)
    # layer outputs are re-rounded to fp16 so accumulation-order differences can flip one rounding per layer
    err = np.abs(got - exp)
    assert (err <= 4 * ulp + 2e-3).mean() > 0.999, f"max err {err.max()}"
    assert np.array_equal(got[:, 3], exp[:, 3]) or (np.abs(got[:, 3] - exp[:, 3]) <= 4 * ulp[:, 3] + 2e-3).all()
