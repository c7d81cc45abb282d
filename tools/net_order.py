"""Sample order vs the fused network kernel: the C3 head launch's NerfCoordinates (lego, 1080p) evaluated in
their wavefront order, Morton orders of the warped position and a random permutation (same samples).
python tools/net_order.py"""
import json
import sys

sys.path.insert(0, "/root/repo")
import numpy as np
import torch

from synerfgine_amd import scene as S

tb, eng, _ = S.make_engine("c3", model="lego")
r = eng.frame()
n = int(r.samples_per_iter[0])
coords = eng.frame_buffer("coords")[: n * 7].reshape(n, 7).copy()


def morton(p, bits):
    q = np.clip((p * (1 << bits)).astype(np.int64), 0, (1 << bits) - 1)
    code = np.zeros(len(p), np.int64)
    for b in range(bits):
        for a in range(3):
            code |= ((q[:, a] >> b) & 1) << (3 * b + a)
    return code


orders = {"wavefront": np.arange(n), "random": np.random.default_rng(0).permutation(n)}
for bits in (4, 6, 8, 10):
    orders[f"morton{bits}"] = np.argsort(morton(coords[:, :3], bits), kind="stable")
out = torch.empty(n * 4, dtype=torch.int16, device="cuda")
st = torch.cuda.current_stream()
res = {"samples": n}
for name, o in orders.items():
    X = torch.from_numpy(np.ascontiguousarray(coords[o])).cuda()
    for _ in range(3):
        tb.inference_mixed_precision(X.data_ptr(), 7, n, out.data_ptr(), 1, st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(20):
        tb.inference_mixed_precision(X.data_ptr(), 7, n, out.data_ptr(), 1, st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    res[name] = {"ms": round(ms, 4), "frac": round(n * 548 / (ms * 1e-3) / 8e12, 4)}
print(json.dumps(res))
tb.close()
