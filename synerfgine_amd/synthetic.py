"""Synthetic 'lego-like' NeRF snapshot content (no datasets or checkpoints are reachable).

Random-init weights of the reference architecture (configs/nerf/base.json:
hash grid L=8, F=4, T=2^19, Nmin=16, b=2 for aabb_scale 1; 64-wide density and
rgb MLPs) with a deterministic analytic density so that rays terminate like a
trained opaque object.  The density signal is injected through the dense
64^3 level (feature 0 = clamped inside-ness of an analytic SDF) and a pair of
ReLU units in the density MLP; everything else is seeded Xavier/uniform noise.
The density grid (snapshot "density_grid_binary", fp16, Morton order) is
derived from the same SDF, dilated by half a cell diagonal.
"""
import numpy as np

L, F, LOG2T, NMIN = 8, 4, 19, 16
PER_LEVEL_SCALE = 2.0  # float(exp(log(2048*aabb_scale/Nmin)/(L-1))) for aabb_scale 1 (testbed.cu:3739)
MIN_STEP = np.float32(np.float32(1.73205080757) / np.float32(1024.0))
GRID = 128


def level_table():
    """tcnn GridEncoding offset table for the lego config (b = 2 -> exact scales)."""
    offsets, res = [0], []
    for l in range(L):
        scale = 2.0 ** l * NMIN - 1.0
        r = int(np.ceil(scale)) + 1
        n = min(((r ** 3 + 7) // 8) * 8, 1 << LOG2T)
        offsets.append(offsets[-1] + n)
        res.append(r)
    return offsets, res


def n_params():
    offsets, _ = level_table()
    return 3072 + 7168 + offsets[-1] * F


SHAPE_SCALE = 1.55
SHAPE_CENTER = np.array([0.5, 0.42, 0.5])


def sdf(p):
    """Signed distance of a lego-ish union of boxes/spheres/capsule in [0,1]^3 (y up)."""
    p = (np.asarray(p, dtype=np.float64) - SHAPE_CENTER) / SHAPE_SCALE + SHAPE_CENTER
    return _sdf_unit(p) * SHAPE_SCALE


def _sdf_unit(p):

    def box(c, h):
        q = np.abs(p - np.asarray(c)) - np.asarray(h)
        return np.linalg.norm(np.maximum(q, 0.0), axis=-1) + np.minimum(q.max(axis=-1), 0.0)

    def sphere(c, r):
        return np.linalg.norm(p - np.asarray(c), axis=-1) - r

    def capsule(a, b, r):
        a, b = np.asarray(a), np.asarray(b)
        pa, ba = p - a, b - a
        h = np.clip((pa @ ba) / (ba @ ba), 0.0, 1.0)
        return np.linalg.norm(pa - h[..., None] * ba, axis=-1) - r

    d = box((0.5, 0.36, 0.5), (0.27, 0.06, 0.19))          # chassis
    d = np.minimum(d, box((0.44, 0.49, 0.5), (0.12, 0.08, 0.14)))   # cabin
    d = np.minimum(d, sphere((0.63, 0.47, 0.5), 0.08))     # engine dome
    d = np.minimum(d, capsule((0.55, 0.55, 0.5), (0.76, 0.70, 0.5), 0.035))  # boom
    for x in (0.31, 0.69):
        for z in (0.33, 0.67):
            d = np.minimum(d, sphere((x, 0.27, z), 0.065))  # wheels
    return d


def _xavier(rng, n_out, n_in, gain=1.0):
    s = gain * np.sqrt(6.0 / (n_in + n_out))
    return rng.uniform(-s, s, size=(n_out, n_in))


def lego_like(seed=1337, ramp=0.012, a=2.6, b=2.3):
    """Returns (config dict, params fp16 [n_params], density_grid fp16 [128^3])."""
    rng = np.random.default_rng(seed)
    # ---- MLPs (nerf_network.h:356-371 order: density, rgb)
    dW0 = _xavier(rng, 64, 32, 0.8)
    dW0[0:2, :] = 0.0
    dW0[0, 8] = a      # level 2 feature 0 -> h0 =  a*s
    dW0[1, 8] = -a     #                   -> h1 = -a*s
    dW1 = _xavier(rng, 16, 64)
    dW1[0, :] = 0.0
    dW1[0, 0], dW1[0, 1] = b, -b   # density logit = a*b*s
    rW0 = _xavier(rng, 64, 32)
    rW1 = _xavier(rng, 64, 64)
    rW2 = _xavier(rng, 16, 64, 2.0)
    mlp = np.concatenate([dW0.ravel(), dW1.ravel(), rW0.ravel(), rW1.ravel(), rW2.ravel()])
    # ---- grid
    offsets, res = level_table()
    grid = rng.uniform(-0.08, 0.08, size=(offsets[-1], F))
    grid[offsets[0]:offsets[1]] = rng.uniform(-0.6, 0.6, size=(offsets[1] - offsets[0], F))
    grid[offsets[1]:offsets[2]] = rng.uniform(-0.4, 0.4, size=(offsets[2] - offsets[1], F))
    r2 = res[2]  # 64, dense; vertex v sits at x = (v - 0.5) / scale
    v = (np.arange(r2) - 0.5) / (r2 - 1.0)
    X, Y, Z = np.meshgrid(v, v, v, indexing="ij")
    pts = np.stack([X, Y, Z], axis=-1)
    s = np.clip(-sdf(pts) / ramp, -1.0, 1.0)
    # dense index = x + y*res + z*res^2  ->  flatten with z slowest
    lvl2 = grid[offsets[2]:offsets[3]]
    lvl2[:, 0] = np.transpose(s, (2, 1, 0)).ravel()
    lvl2[:, 1:] = rng.uniform(-0.5, 0.5, size=(lvl2.shape[0], F - 1))
    params = np.concatenate([mlp, grid.ravel()]).astype(np.float16)
    assert params.size == n_params()
    # ---- density grid: sigma * STEPSIZE at Morton-ordered cell centres (max over the cell)
    c = (np.arange(GRID) + 0.5) / GRID
    CX, CY, CZ = np.meshgrid(c, c, c, indexing="ij")
    half_diag = np.sqrt(3.0) / GRID / 2.0
    d = sdf(np.stack([CX, CY, CZ], axis=-1)) - half_diag
    sig = np.exp(a * b * np.clip(-d / ramp, -1.0, 1.0)) * MIN_STEP
    xi, yi, zi = np.meshgrid(np.arange(GRID), np.arange(GRID), np.arange(GRID), indexing="ij")
    morton = _morton3d(xi.ravel(), yi.ravel(), zi.ravel())
    dg = np.zeros(GRID ** 3, dtype=np.float32)
    dg[morton] = sig.ravel()
    cfg = dict(n_levels=L, n_features_per_level=F, log2_hashmap_size=LOG2T, base_resolution=NMIN,
               per_level_scale=PER_LEVEL_SCALE, aabb_scale=1)
    return cfg, params, dg.astype(np.float16)


def _expand_bits(v):
    v = v.astype(np.uint64)
    v = (v * 0x00010001) & 0xFF0000FF
    v = (v * 0x00000101) & 0x0F00F00F
    v = (v * 0x00000011) & 0xC30C30C3
    v = (v * 0x00000005) & 0x49249249
    return v


def _morton3d(x, y, z):
    return (_expand_bits(x) | (_expand_bits(y) << 1) | (_expand_bits(z) << 2)).astype(np.int64)


# ---------------------------------------------------------------------------------------------
# 'kitchen-like' snapshot for config C4: aabb_scale 16 -> m_aabb = [-7.5, 8.5]^3, max_cascade 4,
# cone_angle_constant 1/256 (testbed_nerf.cu:3069-3085).  Exercises the cascaded, exponential-step
# marcher (the general advance_to_occupied path).  b = float(exp(log(2048*16/16)/7)) = 0x403E350F.
# ---------------------------------------------------------------------------------------------
KITCHEN_AABB_SCALE = 16
KITCHEN_PER_LEVEL_SCALE = float(np.array([0x403E350F], np.uint32).view(np.float32)[0])
KITCHEN_CASCADES = 5


def kitchen_level_table():
    """Offsets / resolutions with the reference's float expressions (only res matters for offsets)."""
    log2b = np.float32(np.log2(np.float32(KITCHEN_PER_LEVEL_SCALE)))
    offsets, res = [0], []
    for l in range(L):
        scale = np.float32(np.float64(np.exp2(np.float32(l) * log2b)) * NMIN - 1.0)
        r = int(np.ceil(scale)) + 1
        offsets.append(offsets[-1] + min(((r ** 3 + 7) // 8) * 8, 1 << LOG2T))
        res.append(r)
    return offsets, res


def kitchen_sdf(p):
    """A room (floor, walls, ceiling) with a table, a cabinet and a bowl, in NeRF coordinates (y up)."""
    p = np.asarray(p, dtype=np.float64)

    def box(c, h):
        q = np.abs(p - np.asarray(c)) - np.asarray(h)
        return np.linalg.norm(np.maximum(q, 0.0), axis=-1) + np.minimum(q.max(axis=-1), 0.0)

    def sphere(c, r):
        return np.linalg.norm(p - np.asarray(c), axis=-1) - r

    d = box((0.5, 0.30, 0.8), (0.9, 0.15, 0.6))                # table top at y = 0.45
    d = np.minimum(d, box((-0.7, 0.2, 1.6), (0.35, 0.9, 0.35)))   # cabinet
    d = np.minimum(d, sphere((0.75, 0.62, 1.0), 0.2))            # bowl
    d = np.minimum(d, box((0.5, -1.2, 0.5), (6.5, 0.2, 6.5)))     # floor
    d = np.minimum(d, box((0.5, 3.4, 0.5), (6.5, 0.2, 6.5)))      # ceiling
    d = np.minimum(d, box((0.5, 1.0, 3.6), (6.5, 2.5, 0.2)))      # back wall
    d = np.minimum(d, box((0.5, 1.0, -3.2), (6.5, 2.5, 0.2)))     # wall behind the camera
    d = np.minimum(d, box((-3.4, 1.0, 0.5), (0.2, 2.5, 6.5)))     # side walls
    d = np.minimum(d, box((4.6, 1.0, 0.5), (0.2, 2.5, 6.5)))
    return d


def kitchen_like(seed=1337, ramp=0.2, a=2.6, b=2.3):
    """Returns (config dict, params fp16, density grid fp16 [5 * 128^3]) for aabb_scale 16."""
    rng = np.random.default_rng(seed)
    lo, size = 0.5 - 0.5 * KITCHEN_AABB_SCALE, float(KITCHEN_AABB_SCALE)
    offsets, res = kitchen_level_table()
    # density from level 1 (dense, 48^3 over the 16-unit box), feature 0 = clamped inside-ness
    dW0 = _xavier(rng, 64, 32, 0.8)
    dW0[0:2, :] = 0.0
    dW0[0, 4] = a
    dW0[1, 4] = -a
    dW1 = _xavier(rng, 16, 64)
    dW1[0, :] = 0.0
    dW1[0, 0], dW1[0, 1] = b, -b
    rW0 = _xavier(rng, 64, 32)
    rW1 = _xavier(rng, 64, 64)
    rW2 = _xavier(rng, 16, 64, 2.0)
    mlp = np.concatenate([dW0.ravel(), dW1.ravel(), rW0.ravel(), rW1.ravel(), rW2.ravel()])
    grid = rng.uniform(-0.08, 0.08, size=(offsets[-1], F))
    grid[offsets[0]:offsets[1]] = rng.uniform(-0.6, 0.6, size=(offsets[1] - offsets[0], F))
    r1 = res[1]
    scale1 = np.float64(np.float32(np.float64(np.exp2(np.float32(1) * np.float32(np.log2(np.float32(KITCHEN_PER_LEVEL_SCALE))))) * NMIN - 1.0))
    v = (np.arange(r1) - 0.5) / scale1              # warped coordinate of dense vertex v
    X, Y, Z = np.meshgrid(v, v, v, indexing="ij")
    pts = np.stack([X, Y, Z], axis=-1) * size + lo
    s = np.clip(-kitchen_sdf(pts) / ramp, -1.0, 1.0)
    lvl1 = grid[offsets[1]:offsets[2]]
    lvl1[:, 0] = np.transpose(s, (2, 1, 0)).ravel()
    lvl1[:, 1:] = rng.uniform(-0.5, 0.5, size=(lvl1.shape[0], F - 1))
    params = np.concatenate([mlp, grid.ravel()]).astype(np.float16)
    # density grid, one 128^3 Morton block per cascade m covering 0.5 +- 2^(m-1)
    xi, yi, zi = np.meshgrid(np.arange(GRID), np.arange(GRID), np.arange(GRID), indexing="ij")
    morton = _morton3d(xi.ravel(), yi.ravel(), zi.ravel())
    dg = np.zeros(KITCHEN_CASCADES * GRID ** 3, dtype=np.float32)
    c = (np.arange(GRID) + 0.5) / GRID
    for m in range(KITCHEN_CASCADES):
        w = 2.0 ** m
        cc = 0.5 + (c - 0.5) * w
        CX, CY, CZ = np.meshgrid(cc, cc, cc, indexing="ij")
        d = kitchen_sdf(np.stack([CX, CY, CZ], axis=-1)) - np.sqrt(3.0) * w / GRID / 2.0
        sig = np.exp(a * b * np.clip(-d / ramp, -1.0, 1.0)) * MIN_STEP
        blk = np.zeros(GRID ** 3, dtype=np.float32)
        blk[morton] = sig.ravel()
        dg[m * GRID ** 3:(m + 1) * GRID ** 3] = blk
    cfg = dict(n_levels=L, n_features_per_level=F, log2_hashmap_size=LOG2T, base_resolution=NMIN,
               per_level_scale=KITCHEN_PER_LEVEL_SCALE, aabb_scale=KITCHEN_AABB_SCALE)
    return cfg, params, dg.astype(np.float16)


def per_level_scale(aabb_scale, n_levels=L, base_resolution=NMIN, desired_resolution=2048.0):
    """Testbed::reset_network's automatic per_level_scale (testbed.cu:3737-3741), in float with glibc's expf / logf:
    exp(log(desired_resolution * aabb_scale / base_resolution) / (n_levels - 1))."""
    import ctypes
    import ctypes.util
    libm = ctypes.CDLL(ctypes.util.find_library("m"))
    libm.expf.restype = libm.logf.restype = ctypes.c_float
    libm.expf.argtypes = libm.logf.argtypes = [ctypes.c_float]
    x = np.float32(np.float32(desired_resolution) * np.float32(aabb_scale) / np.float32(base_resolution))
    return float(libm.expf(np.float32(np.float32(libm.logf(x)) / np.float32(n_levels - 1))))


def random_init(seed=1337, cfg=None, aabb_scale=1):
    """Freshly initialised base.json network (tcnn: hash-grid entries U(-1e-4, 1e-4), Xavier-uniform
    MLP weights) -- the starting point of online training.  `aabb_scale` > 1 (a real capture such as fox):
    the per_level_scale reset_network derives for it, and the grid sized by the library's level table."""
    rng = np.random.default_rng(seed)
    mlp = np.concatenate([_xavier(rng, 64, 32).ravel(), _xavier(rng, 16, 64).ravel(), _xavier(rng, 64, 32).ravel(), _xavier(rng, 64, 64).ravel(),
                          _xavier(rng, 16, 64).ravel()])
    if cfg is None:
        pls = PER_LEVEL_SCALE if aabb_scale == 1 else per_level_scale(aabb_scale)
        cfg = dict(n_levels=L, n_features_per_level=F, log2_hashmap_size=LOG2T, base_resolution=NMIN, per_level_scale=pls, aabb_scale=aabb_scale)
    if cfg.get("aabb_scale", 1) == 1 and cfg.get("per_level_scale") == PER_LEVEL_SCALE:
        offsets, _ = level_table()
        n_grid = offsets[-1] * F
    else:   # the library's GridEncoding level table (sng_nerf_param_count)
        from . import _lib
        n_grid = int(_lib.load().sng_nerf_param_count(_lib.sng_nerf_config(**cfg))) - 10240
    grid = rng.uniform(-1e-4, 1e-4, size=n_grid)
    return cfg, np.concatenate([mlp, grid]).astype(np.float16)
