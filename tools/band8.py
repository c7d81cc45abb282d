"""Thin-band (8-way) frame cost under engine overrides: max over balanced bands of the wall time,
with the raytrace / NeRF stage split of the slowest band.  python tools/band8.py [N]"""
import json
import sys
import time

sys.path.insert(0, "/root/repo")
import torch

from synerfgine_amd import scene as S
from synerfgine_amd.tiling import balance_bounds, even_bounds

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
tb, eng, _ = S.make_engine("c3", model="lego")
H = eng.resolution()["mesh"][1]


def t_frame(rows, reps=5):
    eng.frame(rows=rows)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = eng.frame(rows=rows)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, r


full, _ = t_frame(None)
b = even_bounds(H, N)
for _ in range(6):
    b = balance_bounds(H, b, [t_frame((b[r], b[r + 1]), reps=2)[0] for r in range(N)])
print(json.dumps({"full_ms": round(full, 3), "bounds": b}), flush=True)
CASES = [{}, {"nerf_fused_after": 0}, {"nerf_fused_blocks": 0}, {"nerf_fused_after": 0, "nerf_fused_blocks": 0}, {"rt_start_chunk": 0},
         {"concurrent_streams": 0}, {"rt_reserved_cus": 32}, {"rt_reserved_cus": 64, "nerf_fused_after": 0}]
if len(sys.argv) > 2:
    CASES = [dict((kv.split("=")[0], float(kv.split("=")[1])) for kv in c.split(",") if kv) for c in sys.argv[2].split(";")]
base = {k: eng.get_param(k) for c in CASES for k in c}
for ov in CASES:
    for k, v in base.items():
        eng.set_param(k, v)
    for k, v in ov.items():
        eng.set_param(k, v)
    res = []
    for r in range(N):
        ms, fr = t_frame((b[r], b[r + 1]))
        res.append((ms, fr.ms_raytrace, fr.ms_nerf, fr.n_iterations))
    worst = max(res)
    print(json.dumps({"overrides": ov, "max_ms": round(worst[0], 3), "pred_eff": round(full / (N * worst[0]), 3),
                      "worst_rt_nerf_iters": [round(worst[1], 3), round(worst[2], 3), worst[3]],
                      "band_ms": [round(x[0], 3) for x in res]}), flush=True)
tb.close()
