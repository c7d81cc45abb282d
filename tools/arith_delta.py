"""What the raytracer's arithmetic model changes in a C3 frame: render the benchmarked 1920x1080
frame (lego snapshot + armadillo, the same RNG states) with a library build and save its layers, then compare two
builds -- the IEEE model (make BUILD=_build_ieee MESH_EXTRA="-ffp-contract=off -DRT_TRI_RCP_EXACT -DRT_IEEE_TRANSCENDENTALS") against the default
fast-math model (FMA contraction, the hardware reciprocal in the triangle test, __logf / __expf in the cascaded shadow marches).
  SNG_LIB_PATH=<lib> python tools/arith_delta.py dump out.npz
  python tools/arith_delta.py cmp ieee.npz fast.npz [out.json]
A pixel whose mesh XORWOW state differs after the frame drew a different number of random numbers: some query of its
path turned from hit to miss (or back) -- a topology flip.  A pixel with equal states but a different mesh depth or
colour took the same path with a different closest hit t (or triangle)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(path):
    from synerfgine_amd import scene as S
    tb, eng, _ = S.make_engine("c3", model="lego" if os.path.exists(S.LEGO_INGP) else "synthetic")
    try:
        n0, m0 = eng.rng_states(0).copy(), eng.rng_states(1).copy()
        r = eng.frame(spp=0, reset=True)
        out = {k: r.download(k) for k in ("final_rgba", "syn_rgba", "syn_depth")}
        out["rng_mesh"] = eng.rng_states(1).copy()
        eng.set_rng_states(0, n0)
        eng.set_rng_states(1, m0)
        eng.set_param("rt_count", 1)
        eng.frame(spp=0, reset=True)
        eng.set_param("rt_count", 0)
        c = eng.rt_counters()
        out["counters"] = np.array([c[k][f] for k in ("path", "shadow") for f in ("queries", "box_tests", "tri_tests")], np.uint64)
    finally:
        tb.close()
    np.savez(path, **out)
    print("wrote", path)


def cmp(a, b, out=None):
    A, B = np.load(a), np.load(b)
    W = A["syn_depth"].shape[1]
    st_a, st_b = A["rng_mesh"], B["rng_mesh"]
    ax = 0 if st_a.shape[0] == 6 and st_a.ndim == 2 and st_a.shape[1] != 6 else -1   # [6][n_px] or [n_px][6]
    flip = (st_a != st_b).any(axis=ax).reshape(-1)
    n_px = flip.size
    hit = (A["syn_depth"] < 1e3).reshape(-1) | (B["syn_depth"] < 1e3).reshape(-1)
    dd = np.abs(A["syn_depth"].astype(np.float64) - B["syn_depth"]).reshape(-1)
    t_only = (~flip) & (dd > 0)
    fa, fb = np.clip(A["final_rgba"][..., :3], 0, 1), np.clip(B["final_rgba"][..., :3], 0, 1)
    err = np.abs(fa - fb)
    mse = float(np.mean(err ** 2))
    res = {"pixels": int(n_px), "pixels_hitting_a_mesh": int(hit.sum()),
           "path_topology_flips": int(flip.sum()), "path_topology_flip_frac_of_mesh_pixels": round(float(flip.sum()) / max(1, int(hit.sum())), 6),
           "same_path_other_hit_t": int(t_only.sum()), "max_depth_delta_same_path": float(dd[t_only].max()) if t_only.any() else 0.0,
           "final_psnr_db": round(10 * np.log10(1.0 / max(mse, 1e-12)), 2), "final_max_abs": round(float(err.max()), 5),
           "final_frac_within_2_255": round(float((err.max(axis=-1) <= 2 / 255).mean()), 6),
           "final_frac_bit_equal": round(float((A["final_rgba"] == B["final_rgba"]).all(axis=-1).mean()), 6),
           "counters": {"a": A["counters"].tolist(), "b": B["counters"].tolist(),
                        "order": ["path queries", "path box tests", "path tri tests", "shadow queries", "shadow box tests", "shadow tri tests"]},
           "width": int(W)}
    print(json.dumps(res))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None)
