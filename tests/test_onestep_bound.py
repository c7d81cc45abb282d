"""The one-step regime's no-death bound (fused.hip os_no_death): pass 0 skips the closed loop of a periodic ray
when the bound says its opacity stays at or below `opaque` for n more iterations of the float recurrence
w' = fl(w + fl(a * fl(1 - w))).  Checked here against that recurrence simulated in float32 (the bound restated
in numpy with the same double-precision expression): it must never claim "no death" for a ray that does pass
the threshold within n iterations, and it must hold for the slowly saturating rays it exists for."""
import numpy as np

U = 5.9604644775390625e-08   # 2^-24


def no_death(w0, amax, n, opaque):
    ar = amax.astype(np.float64) * (1.0 + 2.0 * U + U * U) * (1.0 + 1e-12)
    ok = ar < 0.5
    ar = np.where(ok, ar, 0.25)
    tn = (1.0 - w0.astype(np.float64)) * np.exp(n * np.log1p(-ar) * (1.0 + 1e-12)) * (1.0 - 1e-12) - 1.0001 * n * U
    return ok & (tn > (1.0 - float(opaque)) * (1.0 + 1e-9) + 1e-15)


def first_death(w0, a, n, opaque):
    """Iteration (0-based) at which the float32 recurrence first passes `opaque`, or n if it does not."""
    w = w0.astype(np.float32).copy()
    a = a.astype(np.float32)
    one = np.float32(1.0)
    died = np.full(w.shape, n, dtype=np.int64)
    for x in range(n):
        w = (w + (a * (one - w)).astype(np.float32)).astype(np.float32)
        newly = (w > opaque) & (died == n)
        died[newly] = x
    return died


def test_bound_is_sound_and_useful():
    opaque = np.float32(1.0) - np.float32(0.01)   # 1 - render_min_transmittance
    rng = np.random.default_rng(7)
    a = np.concatenate([10.0 ** rng.uniform(-8, -0.4, 6000), 10.0 ** np.linspace(-8, -0.4, 400)]).astype(np.float32)
    w0 = np.concatenate([rng.uniform(0, 0.989, 6000), np.full(400, 0.5)]).astype(np.float32)
    w0 = np.minimum(w0, opaque)
    n = 1200
    died = first_death(w0, a, n, opaque)
    for horizon in (1, 7, 64, 300, 1200):
        claim = no_death(w0, a, horizon, opaque)
        wrong = claim & (died < horizon)
        assert not wrong.any(), f"bound claims no death within {horizon} for a={a[wrong][:3]}, w0={w0[wrong][:3]}"
    # useful: most rays that survive the whole span are recognised (the ones the closed loop spent its time on)
    survive = died >= n
    claim = no_death(w0, a, n, opaque)
    assert claim[survive].mean() > 0.9
