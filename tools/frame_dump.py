"""Render fixed-seed frames of C3 and C4 (full frame + a band) and save every output buffer, for bit-exact A/B of
two library builds: SNG_LIB_PATH=<lib> python tools/frame_dump.py out.npz; then python tools/frame_dump.py --cmp a.npz b.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(path):
    from synerfgine_amd import scene as S
    out = {}
    for cfg, w, h, ov in (("c3", 480, 270, {}), ("c3", 480, 270, {"nerf_shadow_samples": 4}), ("c4", 480, 270, {})):
        tb, eng, _ = S.make_engine(cfg, width=w, height=h, overrides=dict(ov, res_factor=2))
        for rows in (None, (100, 171)):
            for f in range(2):
                r = eng.frame(rows=rows)
                for k in ("final_rgba", "nerf_rgba", "syn_rgba", "syn_depth"):
                    out[f"{cfg}_{len(ov)}_{rows}_{f}_{k}"] = r.download(k)
        out[f"{cfg}_{len(ov)}_rng0"] = eng.rng_states(0).copy()
        out[f"{cfg}_{len(ov)}_rng1"] = eng.rng_states(1).copy()
        tb.close()
    np.savez(path, **out)
    print("wrote", path, len(out), "arrays")


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = [k for k in A.files if not np.array_equal(A[k].view(np.uint32) if A[k].dtype.itemsize == 4 else A[k], B[k].view(np.uint32) if B[k].dtype.itemsize == 4 else B[k])]
    print("arrays", len(A.files), "differing", len(bad), bad[:8])
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "--cmp":
        sys.exit(cmp(sys.argv[2], sys.argv[3]))
    dump(sys.argv[1])
