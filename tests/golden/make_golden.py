"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py            # rewrites tests/golden/*.npz

The reference ships no golden vectors (no tests, tiny-cuda-nn and cuRAND
unvendored, not compilable here), so these fixtures are produced by the oracle after it was
pinned by tests/test_oracle_kat.py (published constants, scipy Sobol, Marsaglia XORWOW,
SURVEY Appendix B) and tests/test_oracle_numpy.py (independent numpy restatement).  They freeze
that state: tests/test_golden.py re-derives them on the CPU, tests/test_gpu_golden.py checks the
HIP path against them on the GPU.  Inputs are seeded (1337) or listed in the file.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

SEED = 1337
L8F4 = dict(n_levels=8, n_features_per_level=4, log2_hashmap_size=19, base_resolution=16, per_level_scale=2.0, aabb_scale=1)
L16F2 = dict(n_levels=16, n_features_per_level=2, log2_hashmap_size=19, base_resolution=16,
             per_level_scale=float(np.array([0x3FB0E285], np.uint32).view(np.float32)[0]), aabb_scale=1)


def random_params(cfg, seed=SEED):
    """Seeded fp16 parameter blob (density MLP, rgb MLP, grid) with O(1) grid values."""
    import oracle as O
    n = O.lib().orc_n_params(O.Model(cfg, np.zeros(1, np.float16)).ref())
    rng = np.random.default_rng(seed)
    p = np.empty(n, np.float16)
    p[:10240] = rng.uniform(-0.25, 0.25, 10240)
    p[10240:] = rng.uniform(-1.0, 1.0, n - 10240)
    return p


def coords(n, seed=SEED):
    rng = np.random.default_rng(seed)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = rng.uniform(0, 1, (n, 3))
    k = n // 8
    c[:k, :3] = rng.integers(0, 2, (k, 3))                       # faces / corners of the unit cube
    c[k:2 * k, :3] = np.float32(1.0) - rng.uniform(0, 1e-6, (k, 3)).astype(np.float32)
    c[:, 3] = rng.uniform(0, 1, n)
    d = rng.normal(size=(n, 3))
    c[:, 4:7] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) * 0.5
    return c


def look_at_camera(view, at, dist):
    """mat4x3 columns (right, down, forward, position) looking along `view` at `at`."""
    f = np.asarray(view, np.float64)
    f /= np.linalg.norm(f)
    up = np.array([0.0, 1.0, 0.0])
    r = np.cross(f, up)
    r /= np.linalg.norm(r)
    dn = np.cross(f, r)
    pos = np.asarray(at) - f * dist
    return np.stack([r, dn, f, pos], 1).astype(np.float32)   # 3x4, column-major when raveled with order="F"


def obj_tris(path):
    v, tris = [], []
    for line in open(path):
        p = line.split()
        if not p:
            continue
        if p[0] == "v":
            v.append([float(a) for a in p[1:4]])
        elif p[0] == "f":
            idx = [int(a.split("/")[0]) - 1 for a in p[1:]]
            for k in range(1, len(idx) - 1):
                tris.append(v[idx[0]] + v[idx[k]] + v[idx[k + 1]])
    return np.array(tris, np.float32)


def gen_rng():
    import ctypes
    import oracle as O
    L = O.lib()
    sob = np.array([[L.orc_sobol(i, d) for d in range(2)] for i in range(256)], np.uint32)
    ldv = np.array([[L.orc_ld_random_val(s, idx * 786433, 0) for s in range(4)] for idx in range(64)], np.float32)
    off = np.zeros((16, 2), np.float32)
    for s in range(16):
        o = (ctypes.c_float * 2)()
        L.orc_ld_random_pixel_offset(s, o)
        off[s] = [o[0], o[1]]
    states = O.xorwow_states(4096)                                   # curand_init(1999, idx, 0)
    draws = np.zeros((8, 16), np.uint32)
    unif = np.zeros((8, 16), np.float32)
    for i in range(8):
        st = states[i].copy()
        st2 = states[i].copy()
        for j in range(16):
            draws[i, j] = L.orc_xorwow_next(O.ptr(st))
            unif[i, j] = L.orc_curand_uniform(O.ptr(st2))
    return dict(sobol=sob, ld_random_val=ldv, pixel_offset=off, xorwow_states=states, xorwow_draws=draws, curand_uniform=unif)


def gen_encode(cfg, n=1024):
    import oracle as O
    p = random_params(cfg)
    c = coords(n)
    m = O.Model(cfg, p)
    enc = O.encode(m, c, 7)
    offs, res = O.level_table(cfg)
    out = dict(coords=c, encoding=enc.view(np.uint16), level_offsets=offs, level_res=res)
    if cfg is L8F4:
        out["network"] = O.inference(m, c[:512]).view(np.uint16)
    return out


def gen_bitfield():
    import hashlib
    import oracle as O
    from synerfgine_amd import synthetic
    _, _, grid = synthetic.lego_like(seed=SEED)
    bf, mean = O.bitfield(grid)
    per_cascade = np.array([int(np.unpackbits(bf[i * 128 ** 3 // 8:(i + 1) * 128 ** 3 // 8]).sum()) for i in range(8)], np.int64)
    return dict(sha256=np.frombuffer(hashlib.sha256(bf.tobytes()).digest(), np.uint8), mean=np.float32(mean),
                popcount_per_cascade=per_cascade, grid_sha256=np.frombuffer(hashlib.sha256(grid.tobytes()).digest(), np.uint8))


def gen_bvh():
    import oracle as O
    tris = obj_tris(os.path.join(REPO, "data", "obj", "armadillo.obj"))
    t2 = tris.copy()
    cap = 4 * len(t2) + 8
    nodes = np.zeros((cap, 8), np.float32)
    n = O.lib().orc_bvh_build(O.ptr(t2), len(t2), 4, O.ptr(nodes), cap)
    nodes = nodes[:n].copy()
    rng = np.random.default_rng(SEED)
    nr = 4096
    lo, hi = t2.reshape(-1, 3).min(0), t2.reshape(-1, 3).max(0)
    tgt = rng.uniform(lo, hi, (nr, 3)).astype(np.float32)
    org = (tgt + rng.normal(size=(nr, 3)) * (hi - lo).max()).astype(np.float32)
    d = tgt - org
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    obj = dict(nodes=nodes, tris=t2, rot=np.eye(3, dtype=np.float32).ravel(order="F"), pos=np.zeros(3, np.float32), scale=1.0, mat_id=0)
    oo = O.make_objects([obj])
    t_out = np.zeros(nr, np.float32)
    o_out = np.zeros(nr, np.int32)
    O.lib().orc_depth_test_world(oo, 1, O.ptr(org), O.ptr(d), nr, O.ptr(t_out), O.ptr(o_out))
    return dict(tris_in=tris, nodes=nodes, tris=t2, ray_o=org, ray_d=d, t=t_out, obj=o_out)


def gen_frame():
    import oracle as O
    from synerfgine_amd import synthetic
    cfg, params, grid = synthetic.lego_like(seed=SEED)
    m = O.Model(cfg, params)
    vol = O.make_volume(O.bitfield(grid)[0])
    W = H = 64
    cam = look_at_camera([0.6119312, -0.104988195, -0.7839119], [0.5, 0.42, 0.5], 1.5)
    focal = 0.5 / np.tan(0.5 * np.deg2rad(50.625)) * H
    c = O.make_camera(cam.ravel(order="F"), (focal, focal), (W, H))
    rgba, depth, pos, nrm, st = O.render_nerf(m, vol, c)
    n_it = st.n_iterations
    return dict(camera=cam.ravel(order="F"), focal=np.float32(focal), rgba=rgba, depth=depth, positions=pos,
                n_iterations=np.int64(n_it), n_samples=np.int64(st.n_samples), n_hit=np.int64(st.n_hit),
                alive_per_iter=np.array(st.alive_per_iter[:n_it], np.int64), steps_per_iter=np.array(st.steps_per_iter[:n_it], np.int64))


GENERATORS = {
    "rng": gen_rng,
    "encode_l8f4": lambda: gen_encode(L8F4),
    "encode_l16f2": lambda: gen_encode(L16F2),
    "bitfield_lego_like": gen_bitfield,
    "bvh_armadillo": gen_bvh,
    "frame_nerf_64": gen_frame,
}


def main(names=None):
    for name, fn in GENERATORS.items():
        if names and name not in names:
            continue
        data = fn()
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **data)
        print(name, {k: getattr(v, "shape", ()) for k, v in data.items()})


if __name__ == "__main__":
    main(sys.argv[1:])
