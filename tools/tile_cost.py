"""How long the path kernel's single tiles take (raytrace_kernel records each 8x8 tile's wall-clock cycles,
s_memrealtime at 100 MHz, into rt_tile_cost).  The slowest tile is a floor for any band split: one wave runs the
tile's 64 pixels x 8 samples x 2 bounces as a chain, whatever the band height.

python tools/tile_cost.py [--config c3] [--bounds 501-560 ...] [--frames 5]
Prints one JSON line per case: the frame (or band) time, the path kernel's stages, and the tile-time quantiles."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from synerfgine_amd import scene as S  # noqa: E402

CLOCK_HZ = 100e6   # s_memrealtime on gfx950

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--bounds", action="append", default=[])
ap.add_argument("--frames", type=int, default=5)
ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
args = ap.parse_args()
model = "lego" if args.config != "c4" else "synthetic"
ov = {kv.split("=")[0]: float(kv.split("=")[1]) for kv in args.set}
tb, eng, _ = S.make_engine(args.config, model=model, overrides=ov)
W, H = eng.resolution()["mesh"]
cases = [None] + [tuple(int(x) for x in b.replace("-", ",").split(",")) for b in args.bounds]
for rows in cases:
    for _ in range(3):
        r = eng.frame(rows=rows) if rows else eng.frame()
    ms = []
    for _ in range(args.frames):
        r = eng.frame(rows=rows, collect_kernel_times=True) if rows else eng.frame(collect_kernel_times=True)
        ms.append(r.ms_raytrace)
    torch.cuda.synchronize()
    y0, y1 = rows if rows else (0, H)
    tw, th = int(eng.get_param("rt_tile")), int(eng.get_param("rt_tile_h")) or int(eng.get_param("rt_tile"))
    n_tiles = ((W + tw - 1) // tw) * ((y1 - y0 + th - 1) // th)
    cost = eng.frame_buffer("rt_tile_cost", np.uint32)[:n_tiles].astype(np.float64) / CLOCK_HZ * 1e3
    q = np.quantile(cost, [0.5, 0.9, 0.99, 0.999, 1.0])
    print(json.dumps({"config": args.config, "rows": [y0, y1], "tiles": n_tiles, "raytrace_ms_median": round(float(np.median(ms)), 3),
                      "tile_ms_quantiles": {k: round(float(v), 4) for k, v in zip(["p50", "p90", "p99", "p999", "max"], q)},
                      "tiles_over_0p5ms": int((cost > 0.5).sum()), "tile_ms_sum": round(float(cost.sum()), 2)}), flush=True)
tb.close()
