"""N-way band split of one frame, measured on ONE GPU: every band of a cost-balanced split is rendered alone
(as its rank would render it, with the frame-wide step schedule the bands share through the per-iteration
alive-count all-reduce), and the slowest band bounds the N-GPU frame.  Prints the full frame's wall time,
the balanced bounds, and per engine-override case: the slowest band, the predicted N-GPU frames/s
(1000 / slowest band, before the RGBA8 gather to rank 0: 4 B/px, ~8 MB per 1080p frame over xGMI) and the
predicted strong-scaling efficiency full / (N x slowest).

usage: python tools/band8.py [--n N] [--config c3|c4] [--cases "k=v+k=v/k=v"] [--model lego|synthetic]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from synerfgine_amd import scene as S  # noqa: E402
from synerfgine_amd.tiling import balance_bounds, even_bounds  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=8)
ap.add_argument("--config", default="c3")
ap.add_argument("--cases", default="")
ap.add_argument("--model", default=None)
args = ap.parse_args()
N = args.n
model = args.model or ("lego" if args.config != "c4" else "synthetic")
tb, eng, _ = S.make_engine(args.config, model=model)
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
print(json.dumps({"config": args.config, "model": model, "n": N, "full_ms": round(full, 3), "full_fps": round(1000.0 / full, 2),
                  "bounds": b}), flush=True)
CASES = [{}]
if args.cases:
    CASES = [dict((kv.split("=")[0], float(kv.split("=")[1])) for kv in c.split("+") if kv) for c in args.cases.split("/")]
base = {k: eng.get_param(k) for c in CASES for k in c}
for ov in CASES:
    for k, v in base.items():
        eng.set_param(k, v)
    for k, v in ov.items():
        eng.set_param(k, v)
    res = []
    for r in range(N):
        ms, fr = t_frame((b[r], b[r + 1]))
        res.append((ms, fr.ms_raytrace, fr.ms_nerf, fr.n_iterations, fr.ms_frame, fr.ms_shadow, fr.network_launches))
    worst = max(res)
    print(json.dumps({"overrides": ov, "max_band_ms": round(worst[0], 3), "pred_fps": round(1000.0 / worst[0], 1),
                      "pred_eff": round(full / (N * worst[0]), 3), "worst_band_rt_nerf_ms_iters": [round(worst[1], 3), round(worst[2], 3), worst[3]],
                      "band_ms": [round(x[0], 3) for x in res],
                      "band_device_frame_nerf_shadow_rt_ms": [[round(x[4], 3), round(x[2], 3), round(x[5], 3), round(x[1], 3)] for x in res],
                      "band_network_launches": [x[6] for x in res]}), flush=True)
tb.close()
