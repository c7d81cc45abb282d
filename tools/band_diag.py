"""Per-band frame times for N-way row tiling (predicts strong-scaling efficiency of bench.py --gpus N)."""
import json
import sys
import time

sys.path.insert(0, "/root/repo")
import torch

from synerfgine_amd import scene as S
from synerfgine_amd.tiling import balance_bounds, band_rows, even_bounds

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
ov = dict((kv.split("=")[0], float(kv.split("=")[1])) for kv in sys.argv[2:])
tb, eng, _ = S.make_engine(cfg, overrides=ov)
H = eng.resolution()["mesh"][1]


def t_frame(rows, reps=5):
    eng.frame(rows=rows)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.frame(rows=rows)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


full = t_frame(None)
out = {"config": cfg, "overrides": ov, "full_ms": round(full, 3)}
for n in (2, 4, 8):
    ts = [round(t_frame(band_rows(H, r, n)), 3) for r in range(n)]
    out[f"n{n}"] = {"band_ms": ts, "max": max(ts), "pred_eff": round(full / (n * max(ts)), 3)}
    b = even_bounds(H, n)
    for _ in range(8):
        tb_ = [t_frame((b[r], b[r + 1]), reps=2) for r in range(n)]
        b = balance_bounds(H, b, tb_)
    tb_ = [round(t_frame((b[r], b[r + 1])), 3) for r in range(n)]
    out[f"n{n}_balanced"] = {"bounds": b, "band_ms": tb_, "max": max(tb_), "pred_eff": round(full / (n * max(tb_)), 3)}
print(json.dumps(out), flush=True)
tb.close()
