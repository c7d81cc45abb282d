"""Kernel timeline of the C5 training step (run under rocprofv3 --kernel-trace): the bench's train leg at 60 steps.
Analyse the trace with tools/train_gaps.py."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
r = bench.train_leg(steps=60, warmup=20)
print(r["steps_per_s"], r["ms_per_step"], flush=True)
