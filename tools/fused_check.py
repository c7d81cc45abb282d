"""Fused-tail exactness / determinism probe: compare nerf outputs for nerf_fused_after values vs the
pure wavefront, and repeat runs.  python tools/fused_check.py [config]"""
import json
import sys

sys.path.insert(0, "/root/repo")
import numpy as np

from synerfgine_amd import scene as S

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
tb, eng, _ = S.make_engine(cfg, width=160, height=90, overrides={"show_virtual_obj": 0, "shadow_on_nerf": 0})
n0 = eng.rng_states(0).copy()


def run(**ov):
    for k, v in ov.items():
        eng.set_param(k, v)
    eng.set_rng_states(0, n0)
    r = eng.frame()
    return r.download("nerf_rgba").copy(), list(r.alive_per_iter)[: r.n_iterations], r.n_samples


ref, alive_ref, ns_ref = run(nerf_fused=0)
for fa in (1, 2, 3, 4, 6):
    outs = [run(nerf_fused=1, nerf_fused_after=fa) for _ in range(2)]
    d = [float(np.abs(o[0] - ref).max()) for o in outs]
    print(json.dumps({"fused_after": fa, "max_diff_vs_wavefront": d, "repeat_equal": bool(np.array_equal(outs[0][0], outs[1][0])),
                      "samples": [o[2] for o in outs], "ref_samples": ns_ref, "alive_ref": alive_ref[:8], "alive": outs[0][1][:8]}), flush=True)
tb.close()
