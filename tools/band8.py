"""N-way band split of one frame, measured on ONE GPU under the frame-wide step schedule the ranks share.

A rank of `bench.py --gpus N` renders its row band with the frame-wide schedule: every reduction point of
trace_alt (testbed_nerf.cu:2180-2190: the alive count each iteration; the one-step regime's and the multi-step
rounds' death histograms) sums the ranks' own-row values over RCCL.  Here the full frame's reduced values are
recorded once (a world-size-1 host reducer), and every band is then rendered with those values replayed at its
reduction points (sng_set_sched_replay: an async copy from pinned memory, no host sync, no communicator), so one
process times each band exactly as its rank would render it (tests/test_gpu_bands.py checks that such a band
equals the single-GPU rows bit for bit).  The slowest band bounds the N-GPU frame.

The communication the replay leaves out is priced, not measured (one GPU cannot measure xGMI): each reduction
is an RCCL all-reduce of <= 40 KB on the NeRF stream, priced at --ar-us (default 25 us, an assumed 8-rank
small-message latency over xGMI), and the final RGBA8 gather to rank 0 (4 B/px) at --gather-gbs per peer link.

Prints the full frame's wall time, the balanced bounds, and per engine-override case the slowest band, the
reductions per frame, the predicted N-GPU frames/s and the predicted strong-scaling efficiency
full / (N x predicted frame).

usage: python tools/band8.py [--n N] [--config c3|c4] [--cases "k=v+k=v/k=v"] [--model lego|synthetic] [--out FILE]"""
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
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--ar-us", type=float, default=25.0, help="assumed latency of one small RCCL all-reduce over xGMI")
ap.add_argument("--gather-gbs", type=float, default=50.0, help="assumed per-link bandwidth of the RGBA8 gather to rank 0")
ap.add_argument("--out", default=None, help="append the JSON lines to this file")
args = ap.parse_args()
N = args.n
model = args.model or ("lego" if args.config != "c4" else "synthetic")
tb, eng, _ = S.make_engine(args.config, model=model)
W, H = eng.resolution()["mesh"]
out = open(args.out, "a") if args.out else None


def emit(d):
    line = json.dumps(d)
    print(line, flush=True)
    if out:
        out.write(line + "\n")
        out.flush()


def timed(rows, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = eng.frame(rows=rows)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, r


def record():
    """The full frame's reduced values: [0] from cleared step hints (the first frame after attaching), [1] the
    steady state (hints from the previous frame, which every later frame repeats)."""
    log = eng.record_schedule()
    recs = []
    for _ in range(3):
        eng.frame()
        recs.append(list(log))
        log.clear()
    eng.detach_comm()
    assert recs[1] == recs[2], "the recorded schedule is not steady from frame to frame"
    return recs[0], recs[1]


def t_band(rows, recs, reps):
    """A band as its rank renders it: the first frame replays the cleared-hint records, the timed ones the
    steady records."""
    eng.set_sched_replay(recs[0])
    eng.frame(rows=rows)
    eng.set_sched_replay(recs[1])
    eng.frame(rows=rows)
    ms, r = timed(rows, reps)
    eng.set_sched_replay(None)
    return ms, r


full, rf = timed(None, args.reps)
full, rf = timed(None, args.reps)
recs = record()
n_red = len(recs[1])
b = even_bounds(H, N)
for _ in range(6):
    b = balance_bounds(H, b, [t_band((b[r], b[r + 1]), recs, 2)[0] for r in range(N)])
emit({"config": args.config, "model": model, "n": N, "full_ms": round(full, 3), "full_fps": round(1000.0 / full, 2),
      "full_iterations": rf.n_iterations, "full_onestep": [rf.onestep_from_iter, rf.onestep_iterations], "full_msr_rounds": rf.msr_rounds,
      "bounds": b, "sched": "frame-wide (replayed)", "reductions_per_frame": n_red,
      "reduction_sizes": sorted(set(r[0] for r in recs[1]))})
CASES = [{}]
if args.cases:
    CASES = [dict((kv.split("=")[0], float(kv.split("=")[1])) for kv in c.split("+") if kv) for c in args.cases.split("/")]
base = {k: eng.get_param(k) for c in CASES for k in c}
for ov in CASES:
    for k, v in base.items():
        eng.set_param(k, v)
    for k, v in ov.items():
        eng.set_param(k, v)
    if ov:
        full, rf = timed(None, args.reps)
        recs = record()
        n_red = len(recs[1])
        for _ in range(6):   # the split balanced for this case's costs
            b = balance_bounds(H, b, [t_band((b[r], b[r + 1]), recs, 2)[0] for r in range(N)])
    res = []
    for r in range(N):
        ms, fr = t_band((b[r], b[r + 1]), recs, args.reps)
        assert fr.sched_reductions == n_red
        res.append((ms, fr.ms_raytrace, fr.ms_nerf, fr.n_iterations, fr.ms_frame, fr.ms_shadow, fr.network_launches, fr.msr_rounds))
    worst = max(res)
    comm_ms = n_red * args.ar_us * 1e-3
    # the gather: rank 0 receives N - 1 bands of ~H/N rows x W x 4 B, each over its own xGMI link
    gather_ms = (H / N) * W * 4 / (args.gather_gbs * 1e9) * 1e3 + args.ar_us * 1e-3
    pred = worst[0] + comm_ms + gather_ms
    emit({"overrides": ov, "n": N, "bounds": b, "full_ms": round(full, 3), "max_band_ms": round(worst[0], 3),
          "reductions_per_frame": n_red, "priced_allreduce_ms": round(comm_ms, 3), "priced_gather_ms": round(gather_ms, 3),
          "pred_frame_ms": round(pred, 3), "pred_fps": round(1000.0 / pred, 1), "pred_eff": round(full / (N * pred), 3),
          "pred_eff_compute_only": round(full / (N * worst[0]), 3),
          "worst_band_rt_nerf_ms_iters": [round(worst[1], 3), round(worst[2], 3), worst[3]],
          "band_ms": [round(x[0], 3) for x in res],
          "band_device_frame_nerf_shadow_rt_ms": [[round(x[4], 3), round(x[2], 3), round(x[5], 3), round(x[1], 3)] for x in res],
          "band_network_launches": [x[6] for x in res], "band_msr_rounds": [x[7] for x in res]})
tb.close()
