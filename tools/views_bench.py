"""bench.py's NeRF-dominated legs alone (nerf_views: C2 at the lego dataset camera, the 1 deg/frame orbits at C2 and
C3, the frame-filling 1080p view), for rocprofv3 runs (tools/gpu.sh profpy): python tools/views_bench.py [frames]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 10
print(json.dumps(bench.nerf_views("lego", frames, 2, cpu_check=False)), flush=True)
