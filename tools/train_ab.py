"""Training A/B: the train leg of bench.py (lego400, batch 2^18, stage timings) under engine-parameter cells, run
alternately.  usage: python tools/train_ab.py PAIRS KEY=V[,KEY=V] KEY=V[,KEY=V]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

pairs = int(sys.argv[1])
cells = [dict(kv.split("=") for kv in c.split(",")) if c != "-" else {} for c in sys.argv[2:]]
for p in range(pairs):
    for ci, cell in enumerate(cells):
        r = bench.train_leg(engine_params={k: float(v) for k, v in cell.items()})
        print(json.dumps({"pair": p, "cell": cell, "steps_per_s": r["steps_per_s"], "stage_ms": r["roofline"].get("stage_ms")}), flush=True)
