"""bench.py's stdout line stays parseable by the driver: built from stub frames (no GPU) through the same
frame_result / compact_line / emit_line functions the timed run uses, the line is one JSON object, it is the last
stdout line, and it stays under bench.LINE_MAX_BYTES (the driver reads an 8 KB stdout tail; round 5's 23.7 KB line
was not parsed).  The worst case carries every leg of round 5's full line plus the maximum of 16 network launches
per frame."""
import argparse
import io
import json
import os
import sys
import types
from contextlib import redirect_stdout

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def _stub_frame(n_launch=2):
    launches = [(1200502.0 / (k + 1), 0.161 / (k + 1)) for k in range(n_launch)]
    return types.SimpleNamespace(
        ms_network=sum(m for _, m in launches), network_launches=n_launch, n_samples_network=int(sum(s for s, _ in launches)),
        n_samples=1270000, n_samples_reused=60000, spec_evals=int(sum(s for s, _ in launches)), spec_exec=int(sum(s for s, _ in launches)),
        msr_evals=0, msr_exec=0, ms_fused_tail=0.65, onestep_field_evals=0, ms_onestep=0.0, network_launch=launches,
        n_reference_slots=1320000, n_iterations=14, fused_from_iter=2, onestep_from_iter=0, onestep_iterations=0, n_hit=60000,
        ms_frame=3.3, ms_raytrace=3.1, ms_nerf=2.9, ms_shadow=0.17, ms_overlay=0.02, spec_rounds=2, msr_rounds=0)


def _args(**kw):
    a = dict(config="c3", steps=20, warmup=3, model="lego", serial_streams=False)
    a.update(kw)
    return argparse.Namespace(**a)


def _full(n_launch=2, legs=True):
    stats = [_stub_frame(n_launch) for _ in range(20)]
    res = {"mesh": (1920, 1080), "nerf": (1920, 1080)}
    full = bench.frame_result(_args(), stats, 0.066, 1, res, [0, 1080], {"backend": None, "world_size": 1}, {}, False, True,
                              "data/lego.ingp")
    if legs:   # every leg of round 5's full driver-format line (23.7 KB), the same shapes the run attaches
        r05 = json.load(open(os.path.join(REPO, "profiles", "r05_bench.json")))
        for k in ("c3_nerf_shadow_r", "bvh", "abm_sweep", "nerf_views", "c4fox", "train", "cpu_baseline", "psnr_vs_oracle"):
            full[k] = r05[k]
        full["roofline"]["uncontended"] = r05["roofline"]["uncontended"]
        full["bvh"]["lane_eff"] = {"path": {"record_loop": 0.31, "tri_loop": 0.54}, "shadow": {"record_loop": 0.56, "tri_loop": 0.81}}
        full["bvh"]["useful_frac"] = {"raytrace_kernel": 0.10, "shadow_rays_kernel": 0.24}
        full["bvh"]["algorithmic_flop_frac"] = {"raytrace_kernel": 0.054, "shadow_rays_kernel": 0.20}
    return full


def test_line_from_stub_frames_is_compact_and_complete():
    full = _full()
    assert len(json.dumps(full)) > 12000   # the full result would not fit the tail
    line = bench.compact_line(full)
    s = json.dumps(line)
    assert len(s) < bench.LINE_MAX_BYTES < 8000
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "config", "roofline", "cpu_baseline", "psnr_vs_oracle", "train", "extras"):
        assert k in line, k
    assert line["metric"] == json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
    rf = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert rf["uncontended"]["frac"] > 0 and isinstance(rf["per_launch"], list)
    assert {"value", "cores", "kind", "cpu_model"} <= set(line["cpu_baseline"])
    assert {"steps_per_s", "frac"} <= set(line["train"])
    assert line["extras"].startswith("profiles/bench_extra_")
    assert line["bvh"]["algorithmic_flop_frac"]["shadow_rays_kernel"] > 0


def test_worst_case_line_fits():
    # 16 network launches per frame (sng_frame_result's per-launch record limit) and every leg present
    line = bench.compact_line(_full(n_launch=16))
    assert len(json.dumps(line)) <= bench.LINE_MAX_BYTES
    assert "value" in line and "roofline" in line and "frac" in line["roofline"]


def test_emitted_line_is_the_last_stdout_line_and_parses():
    line = bench.compact_line(_full())
    buf = io.StringIO()
    with redirect_stdout(buf):
        print("some earlier output")
        bench.emit_line(line)
    last = buf.getvalue().rstrip("\n").split("\n")[-1]
    d = json.loads(last)
    assert d["value"] == line["value"] and d["unit"] == "frames/s"


def test_headline_without_legs():
    # --no-sweep / --no-cpu-baseline: the contract keys alone
    line = bench.compact_line(_full(legs=False))
    json.loads(json.dumps(line))
    assert "cpu_baseline" not in line and line["value"] > 0


def test_line_for_a_synthetic_model_without_snapshot():
    # config c4 renders the synthetic kitchen-like model (no .ingp): no snapshot path to report
    stats = [_stub_frame() for _ in range(3)]
    full = bench.frame_result(_args(config="c4", steps=3, model="synthetic"), stats, 0.01, 1, {"mesh": (1920, 1080), "nerf": (1920, 1080)},
                              [0, 1080], {}, {}, False, True, None)
    line = bench.compact_line(full)
    assert line["data"].startswith("synthetic") and line["metric"] == bench.METRICS["c4"]
