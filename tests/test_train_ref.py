"""CPU checks of the online-training references (config 5): the pcg32 restatement against the PCG
reference output, the oracle's generate / Adam against independent restatements, and the torch
reference's loss gradient against the reference's closed form (testbed_nerf.cu:1209-1275)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")


def test_pcg32_known_answer():
    """pcg32_srandom(42, 54) -> O'Neill's pcg32-demo sequence (tcnn pcg32 uses the same seeding)."""
    import train_ref as R
    r = R.Pcg32(42, 54)
    assert [r.next_uint() for _ in range(6)] == [0xA15C02B7, 0x7B47F409, 0xBA1D3330, 0x83D2F293, 0xBFA4784B, 0xCBED606E]


def test_pcg32_advance_equals_stepping():
    import train_ref as R
    a, b = R.Pcg32(1337), R.Pcg32(1337)
    for k in (0, 1, 7, 16, 1000):
        a2, b2 = a.copy(), b.copy()
        a2.advance(k)
        for _ in range(k):
            b2.next_uint()
        assert a2.state == b2.state


def _toy_dataset(n=3, w=24, h=20, seed=0):
    rng = np.random.default_rng(seed)
    imgs = rng.integers(0, 256, (n, h, w, 4), dtype=np.uint8)
    imgs[0, :4, :4] = [0xFF, 0x00, 0xFF, 0x00]   # masked texels
    from synerfgine_amd import nerf_data
    xf = nerf_data.orbit_cameras(n, radius=1.3)
    focal = np.full((n, 2), 30.0, np.float32)
    pp = np.full((n, 2), 0.5, np.float32)
    return imgs, xf, focal, pp


def test_oracle_generate_rays_follow_pcg32(oracle_lib):
    """Rays of orc_train_generate: image by ray index, pixel centre from the first two pcg32 draws after
    advance(16 i), pinhole direction (nerf_device.cuh:553-598, common_device.cuh:403-470)."""
    import train_ref as R
    O = oracle_lib
    imgs, xf, focal, pp = _toy_dataset()
    bf = np.full(128 ** 3 // 8 * 8, 0xFF, np.uint8)
    vol = O.make_volume(bf, aabb_scale=1)
    rng = R.step_rng(1337, 3)
    n_rays = 64
    ns, rays, co = O.train_generate(vol, imgs, xf, focal, pp, rng.state, rng.inc, n_rays, max_per_ray=8)
    n, h, w = imgs.shape[:3]
    for i in range(n_rays):
        r = rng.copy()
        r.advance(16 * i)
        img = (i * n // n_rays) % n
        px = min(max(int(np.float32(r.next_float()) * np.float32(w)), 0), w - 1)
        py = min(max(int(np.float32(r.next_float()) * np.float32(h)), 0), h - 1)
        if tuple(imgs[img, py, px]) == (0xFF, 0x00, 0xFF, 0x00):
            assert ns[i] == 0
            continue
        u, v = (px + 0.5) / w, (py + 0.5) / h
        d = xf[img][:, :3] @ np.array([(u - 0.5) * w / 30.0, (v - 0.5) * h / 30.0, 1.0])
        np.testing.assert_allclose(rays[i, 3:], d, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(rays[i, :3], xf[img][:, 3], rtol=0, atol=0)
        assert ns[i] > 0   # full occupancy: every ray that enters the unit cube gets samples
        c = co[i, : min(8, ns[i])]
        assert (c[:, :3] >= 0).all() and (c[:, :3] <= 1).all()
        np.testing.assert_allclose(c[:, 4:7] * 2 - 1, np.tile(d / np.linalg.norm(d), (len(c), 1)), atol=1e-6)


def test_oracle_adam_ema_vs_numpy(oracle_lib):
    rng = np.random.default_rng(1)
    n, n_matrix = 5000, 1000
    master = rng.normal(size=n).astype(np.float32)
    grads = (rng.normal(size=n) * 100).astype(np.float32)
    grads[3000:3500] = 0
    m1 = (rng.normal(size=n) * 1e-2).astype(np.float32)
    m2 = np.abs(rng.normal(size=n) * 1e-3).astype(np.float32)
    steps = rng.integers(0, 50, n).astype(np.uint32)
    ema = master + np.float32(0.01)
    exp = [a.copy() for a in (master, m1, m2, steps, ema)]
    oracle_lib.train_adam_ema(master, grads, m1, m2, steps, ema, n_matrix=n_matrix, ema_step=7)
    w, f1, f2, st, e = exp
    f = np.float32
    g = grads / f(128.0)
    upd = (np.arange(n) < n_matrix) | (g != 0)
    g = np.where(np.arange(n) < n_matrix, g + f(1e-6) * w, g).astype(np.float32)
    f1n = (f(0.9) * f1 + (f(1) - f(0.9)) * g).astype(np.float32)
    f2n = (f(0.99) * f2 + (f(1) - f(0.99)) * (g * g)).astype(np.float32)
    stn = st + 1
    lr = (f(1e-2) * (np.sqrt(f(1) - np.power(f(0.99), stn.astype(np.float32))) / (f(1) - np.power(f(0.9), stn.astype(np.float32))))).astype(np.float32)
    wn = (w - (lr / (np.sqrt(f2n) + f(1e-15))) * f1n).astype(np.float32)
    w = np.where(upd, wn, w)
    np.testing.assert_array_equal(steps, np.where(upd, stn, st))
    np.testing.assert_allclose(m1, np.where(upd, f1n, f1), rtol=1e-6)
    np.testing.assert_allclose(m2, np.where(upd, f2n, f2), rtol=1e-6)
    np.testing.assert_allclose(master, w, rtol=1e-6)
    do, dn = f(1) - np.power(f(0.95), f(7)), f(1) - np.power(f(0.95), f(8))
    np.testing.assert_allclose(ema, (e * f(0.95) * do + w * (f(1) - f(0.95))) / dn, rtol=1e-6)


def test_loss_gradient_closed_form_equals_autograd():
    """compute_loss_kernel_train_nerf's closed-form dL/d(output) (testbed_nerf.cu:1209-1275) is the
    derivative the torch reference takes by autograd."""
    import train_ref as R
    rng = np.random.default_rng(3)
    for trial in range(20):
        n = int(rng.integers(1, 40))
        out = rng.normal(size=(n, 4)) * [2, 2, 2, 3]
        dt = np.full(n, np.sqrt(3) / 1024) * rng.uniform(1, 4, n)
        tgt, bg = rng.uniform(0, 1, 3), rng.uniform(0, 1, 3)
        cn, loss, g = R.ray_loss_grad(out, dt, tgt, bg, n_rays=1, loss_scale=1.0)
        # closed form
        rgb = 1 / (1 + np.exp(-out[:, :3]))
        alpha = 1 - np.exp(-np.exp(out[:, 3]) * dt)
        T, acc = 1.0, np.zeros(3)
        m = 0
        for j in range(n):
            if T < 1e-4:
                break
            acc += alpha[j] * T * rgb[j]
            T *= 1 - alpha[j]
            m += 1
        if m == n:
            acc += T * bg
        d = acc - tgt
        lg = np.where(np.abs(d) > 0.1, np.sign(d), d / 0.1) / 5.0
        T, acc2 = 1.0, np.zeros(3)
        exp = np.zeros((m, 4))
        for j in range(m):
            w = alpha[j] * T
            acc2 += w * rgb[j]
            T *= 1 - alpha[j]
            suffix = acc - acc2
            exp[j, :3] = w * lg * rgb[j] * (1 - rgb[j])
            exp[j, 3] = np.exp(np.clip(out[j, 3], -15, 15)) * dt[j] * np.dot(lg, T * rgb[j] - suffix)
        assert cn == m
        np.testing.assert_allclose(g, exp, rtol=1e-9, atol=1e-12)


def test_torch_network_matches_oracle(oracle_lib):
    """The torch reference's forward agrees with the oracle's NerfNetwork restatement (fp16 outputs)."""
    import train_ref as R
    from synerfgine_amd import synthetic
    cfg, params = synthetic.random_init(5)
    p = params.copy()
    rng = np.random.default_rng(2)
    p[10240:] = rng.uniform(-1, 1, len(p) - 10240).astype(np.float16)
    c = rng.uniform(0, 1, (500, 7)).astype(np.float32)
    exp = oracle_lib.inference(oracle_lib.Model(cfg, p), c)[:, :4].astype(np.float64)   # rows r, g, b, sigma
    rgb, sig = R.TorchNetwork(cfg, p).forward(c)
    got = np.concatenate([rgb.detach().numpy(), sig.detach().numpy()[:, None]], 1)
    err = np.abs(got - exp)
    assert (err <= 8 * np.spacing(np.abs(exp).astype(np.float16)).astype(np.float64) + 2e-3).all(), err.max()
