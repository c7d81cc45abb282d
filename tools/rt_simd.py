"""SIMD efficiency of the BVH traversal loops (C3 by default): one counting frame with rt_count = 1 (lane-level
box / triangle tests) and one with rt_count = 2 (wave iterations of the record and triangle loops, bvh_walk_near).
efficiency = lane work / (64 x wave iterations).  usage: python tools/rt_simd.py [config] [k=v ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from synerfgine_amd import scene as S
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    overrides = {}
    for kv in sys.argv[2:]:
        k, v = kv.split("=", 1)
        overrides[k] = float(v)
    tb, eng, _ = S.make_engine(cfg, device_id=0, overrides=overrides, model="lego" if os.path.exists(S.LEGO_INGP) else "synthetic")
    for _ in range(3):
        eng.frame(spp=0, reset=True)
    out = {}
    for mode in (1, 2):
        eng.set_param("rt_count", mode)
        eng.frame(spp=0, reset=True)
        out[mode] = eng.rt_counters()
    eng.set_param("rt_count", 0)
    res = {}
    for k in ("path", "shadow"):
        lane, wave = out[1][k], out[2][k]
        res[k] = {"queries": lane["queries"], "box_tests": lane["box_tests"], "tri_tests": lane["tri_tests"],
                  "record_wave_iters": wave["box_tests"], "tri_wave_iters": wave["tri_tests"],
                  "record_loop_eff": round(lane["box_tests"] / 2 / max(1, 64 * wave["box_tests"]), 4),
                  "tri_loop_eff": round(lane["tri_tests"] / max(1, 64 * wave["tri_tests"]), 4)}
    print(json.dumps(res))
    tb.close()


if __name__ == "__main__":
    main()
