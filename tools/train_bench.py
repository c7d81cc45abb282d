"""BASELINE config C5 alone: bench.py's training leg (lego400, batch 2^18, fresh init), for rocprofv3 runs
(tools/gpu.sh profpy / pmcpy): python tools/train_bench.py [steps] [warmup]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 50
print(json.dumps(bench.train_leg(steps, warmup)), flush=True)
