"""Where one path-kernel tile's chain goes: per-tile phase times from the RT_CHAIN_PROBE timing build
(make BUILD=_build_probe EXTRA=-DRT_CHAIN_PROBE; run with SNG_LIB_PATH=synerfgine_amd/_build_probe/libsng_hip.so).
For the slowest tiles of each case: the tile's wall time, the world queries' share, the deferred shading's share, the
record-allocation atomic alone (its wait also drains the wave's pending stores) and the number of queries (lane 0); with
--set rt_count=1 (rt_count=2: wave iterations) also lane 0's box and triangle tests of the tile.

python tools/chain_probe.py [--config c3] [--bounds 540-548 ...] [--set KEY=VALUE ...] [--top 8]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from synerfgine_amd import scene as S  # noqa: E402

TICK_MS = 1e3 / 100e6   # s_memrealtime: 100 MHz

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--bounds", action="append", default=[])
ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
ap.add_argument("--top", type=int, default=8)
args = ap.parse_args()
assert "_build_probe" in os.environ.get("SNG_LIB_PATH", ""), "needs the RT_CHAIN_PROBE build (SNG_LIB_PATH)"
ov = {kv.split("=")[0]: float(kv.split("=")[1]) for kv in args.set}
ov.setdefault("concurrent_streams", 0)
tb, eng, _ = S.make_engine(args.config, model="lego" if args.config != "c4" else "synthetic", overrides=ov)
W, H = eng.resolution()["mesh"]
for rows in [None] + [tuple(int(x) for x in b.split("-")) for b in args.bounds]:
    for _ in range(4):
        r = eng.frame(rows=rows, collect_kernel_times=True) if rows else eng.frame(collect_kernel_times=True)
    torch.cuda.synchronize()
    y0, y1 = rows if rows else (0, H)
    tw, th = int(eng.get_param("rt_tile")), int(eng.get_param("rt_tile_h")) or int(eng.get_param("rt_tile"))
    n = ((W + tw - 1) // tw) * ((y1 - y0 + th - 1) // th)
    buf = eng.frame_buffer("rt_tile_cost", np.uint32)
    cost = buf[:n].astype(np.float64) * TICK_MS
    ph = buf[n:n + 8 * n].reshape(n, 8).astype(np.float64)
    top = np.argsort(-cost)[: args.top]
    rowsout = []
    for t in top:
        q, sh, al, nq = ph[t, 0] * TICK_MS, ph[t, 1] * TICK_MS, ph[t, 2] * TICK_MS, int(ph[t, 3])
        cnt = {"lane0_queries": int(ph[t, 4]), "lane0_box_tests": int(ph[t, 5]), "lane0_tri_tests": int(ph[t, 6])}
        rowsout.append({"tile": int(t), "ms": round(cost[t], 4), "queries_ms": round(q, 4), "shading_ms": round(sh, 4), "alloc_ms": round(al, 4),
                        "rest_ms": round(cost[t] - q - sh, 4), "queries": nq, "us_per_query": round(1e3 * q / max(nq, 1), 2), **cnt})
    print(json.dumps({"config": args.config, "rows": [y0, y1], "tile": [tw, th], "tiles": n, "raytrace_ms": round(r.ms_raytrace, 3),
                      "overrides": ov, "slowest": rowsout}), flush=True)
tb.close()
