#!/usr/bin/env python3
"""bench.py -- rendered frames/s at 1920x1080 (lego .ingp snapshot + armadillo scene, shadows both ways).

One step = one complete Engine::frame (raytrace + NeRF march/encode/MLP/composite +
shadows on the NeRF + overlay) of BASELINE.json config C3.  With N ranks the frame
is split into N horizontal bands (one per GPU, halo rows recomputed) and the final
bands are all-gathered as RGBA8 over RCCL, so the whole job still produces one frame
per step (strong scaling).

`python bench.py --gpus N` without a torch.distributed environment starts the N ranks itself
(torch.distributed.run, one process per GPU) before anything touches the GPU; under torchrun
(WORLD_SIZE set) it runs as one of the ranks and checks that WORLD_SIZE == N.

Prints ONE JSON line on rank 0 (driver contract).
"""
import argparse
import json
import os
import platform
import socket
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BYTES_PER_SAMPLE = 28 + 8 * 8 * 4 * 2 + 8   # NerfCoordinate read + 8 levels x 8 corners x F=4 fp16 + rgb/sigma fp16 write
FLOPS_PER_SAMPLE = 20480                     # 2*(32*64+64*16) + 2*(32*64+64*64+64*16)
HBM_PEAK_GBS = 8000.0                        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_F16_PEAK_TFLOPS = 2500.0                # dense fp16/bf16 MFMA
# FP32 operations of one BVH box test and one triangle test as the reference writes them (every add, multiply,
# division, min/max and compare = 1): BoundingBox::ray_intersect (bounding_box.cuh:163-211: 6 subtractions,
# 6 divisions, 3 swaps as min/max pairs 6, 4 early-out compares, 4 min/max of the candidates = 26) and
# Triangle::ray_intersect (triangle.cuh:45-59: 3 vector subtractions 9, 2 crosses 18, 4 dots 20, 1 division,
# 3 scalings by d, u + v, 5 compares = 57), priced against the FP32 vector peak (MI355X_MICROARCH.md: 157.3 TFLOP/s,
# which counts an FMA as 2)
BOX_TEST_OPS = 26
TRI_TEST_OPS = 57
FP32_VECTOR_PEAK_TFLOPS = 157.3
ROUND = "r06"
EXTRAS_FILE = f"profiles/bench_extra_{ROUND}.json"   # the legs of this build (bench.py --extras), committed
LINE_MAX_BYTES = 6000                        # the driver reads the line from an 8 KB stdout tail

WORKLOADS = {
    "c2": "lego NeRF only (show_virtual_obj=0, shadows off)",
    "c3": "lego NeRF + armadillo.json (light_samples 8, path_trace_depth 2, shadow_on_nerf + shadow_on_virtual_obj)",
    "c4": "kitchen-like NeRF (aabb_scale 16, 5 cascades, cone stepping) + kitchen-rocks.json (bunny/rock/box, light_samples 4, "
          "nerf_shadow_samples 4)",
    "c4fox": "C4's workload on a trained cascaded field: the reference's real fox capture (aabb_scale 4, 3 cascades, cone stepping, "
             "trained here by tools/train_fox.py) + bunny/rock/box (scenes/fox-rocks.json: kitchen-rocks.json's meshes, materials and "
             "rendering keys), light_samples 4, nerf_shadow_samples 4",
    "foxarm": "the reference's own scene for its fox capture (scenes/fox-armadillo.json = scripts/virtual_desc/fox-armadillo.json): "
              "trained fox .ingp (aabb_scale 4, 3 cascades, cone stepping) + bunny + armadillo, a point and a directional light, "
              "light_samples 8, path_trace_depth 2, nerf_on_nerf_shadow_threshold 0.942",
}
METRICS = {
    "c2": "rendered frames/sec at 800x800 (lego .ingp, NeRF only); PSNR vs ref",
    "c3": "rendered frames/sec at 1920\u00d71080 (lego .ingp + 1 mesh); PSNR vs ref",   # BASELINE.json's metric, verbatim
    "c4": "rendered frames/sec at 1920x1080 (kitchen-like .ingp + 3 meshes, light_samples 4); PSNR vs ref",
    "c4fox": "rendered frames/sec at 1920x1080 (trained fox .ingp + 3 meshes, light_samples 4); PSNR vs ref",
    "foxarm": "rendered frames/sec at 1920x1080 (trained fox .ingp + fox-armadillo.json); PSNR vs ref",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4", "c4fox", "foxarm"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sweep", action="store_true", help="skip every leg after the timed region (serialized roofline, BVH "
                                                            "counters, training)")
    ap.add_argument("--extras", default=None, metavar="PATH",
                    help="also run the extra legs (C3 nerf_shadow_samples r=2, the reference's dmrf-compare-abm sweep, the "
                         "NeRF views, the trained-fox C4 legs) and write the full result to PATH (the stdout line stays compact)")
    ap.add_argument("--cpu-runs", type=int, default=5, help="timed oracle runs per CPU-baseline leg (median reported)")
    ap.add_argument("--serial-streams", action="store_true", help="run raytracer and NeRF back to back (profiling)")
    ap.add_argument("--cpu-baseline-scale", type=float, default=1.0, help="the C3-sample leg renders the frame at 1/scale linear resolution")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"], help="gloo: CPU-side gather (rehearsal on one GPU)")
    ap.add_argument("--dry-run", action="store_true", help="form the ranks and exchange the world size only (no GPU; CPU tests)")
    ap.add_argument("--even-bands", action="store_true", help="equal-height bands instead of cost-balanced ones")
    ap.add_argument("--local-schedule", action="store_true",
                    help="N>1: step each band from its own alive count (no per-iteration count all-reduce; not bit-identical to N=1)")
    ap.add_argument("--balance-iters", type=int, default=8, help="untimed calibration frames for the band split")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE", help="engine parameter override (sng_set_param)")
    ap.add_argument("--model", default=None,
                    help="lego (trained .ingp, data/lego.ingp; default for c2/c3 when present), synthetic, or an .ingp path")
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args):
    """--gpus N outside torch.distributed: start N ranks, one process per GPU, with torch.distributed.run as
    a child process.  This parent never initialises the GPU (no torch.cuda / HIP call happens before the
    children exist), and it exits with the launcher's status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def cpu_info():
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:   # cgroup v2 CPU quota (the GPU box grants a share of the host's CPUs; nproc shows them all)
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": quota,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cpu_model": model}


def cpu_baseline_c1(model_name, runs):
    """the reference has no CPU inference path, so the baseline is the oracle (C++ OpenMP,
    -O2, IEEE fp32 -- the CPU restatement of the render path) rendering config C1: one Engine::frame of the
    lego snapshot at 256x256, NeRF only, no virtual objects.  1 warm-up, then the median of `runs` timed
    frames, on all the OpenMP threads the process has and on 1 thread."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from synerfgine_amd import scene as S

    tb, eng, (ncfg, params, grid) = S.make_engine("c2", width=256, height=256, model=model_name)
    try:
        model = O.Model(ncfg, params)
        vol = O.volume_for(ncfg, grid)
        nrng, mrng = eng.rng_states(0).copy(), eng.rng_states(1).copy()
        lib = O.lib()
        all_threads = lib.orc_num_threads()
        legs = {}
        for threads in (all_threads, 1):
            lib.orc_set_num_threads(threads)
            O.render_frame(model, vol, tb, eng, nrng.copy(), mrng.copy())
            ts = []
            for _ in range(runs):
                t0 = time.perf_counter()
                out = O.render_frame(model, vol, tb, eng, nrng.copy(), mrng.copy())
                ts.append(time.perf_counter() - t0)
            med = statistics.median(ts)
            n = int(out["stats"].n_samples)
            legs[threads] = {"threads": threads, "median_s": round(med, 4), "runs_s": [round(t, 4) for t in ts],
                             "frames_per_s": round(1.0 / med, 3), "samples": n, "samples_per_s": round(n / med, 1),
                             "algorithmic_GB_per_s": round(n * BYTES_PER_SAMPLE / med / 1e9, 3)}
        lib.orc_set_num_threads(all_threads)
    finally:
        tb.close()
    return legs, all_threads


def cpu_sample_c3(eng_cfg, config, scale, model_name, overrides):
    """Time the CPU oracle (test infrastructure) on a bounded sample of the benchmarked workload, and compare
    the GPU's frame of that same sample with it (the metric's "PSNR vs ref": the oracle is the reference
    restatement).  Returns (sample, psnr_vs_oracle)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle as O
    from synerfgine_amd import scene as S

    ncfg, params, grid = eng_cfg
    full = S.CONFIGS[config]
    w, h = int(round(full["width"] / scale)), int(round(full["height"] / scale))
    tb, eng, _ = S.make_engine(config, width=w, height=h, model=model_name, overrides=overrides)
    model = O.Model(ncfg, params)
    vol = O.volume_for(ncfg, grid)
    nrng = eng.rng_states(0).copy()
    mrng = eng.rng_states(1).copy()
    gpu = eng.frame(spp=0, reset=True).download("final_rgba")
    t0 = time.perf_counter()
    ref = O.render_frame(model, vol, tb, eng, nrng, mrng)
    dt = time.perf_counter() - t0
    tb.close()
    frac = (w * h) / float(full["width"] * full["height"])
    err = np.abs(np.clip(gpu[..., :3], 0, 1) - np.clip(ref["final"][..., :3], 0, 1))
    mse = float(np.mean(err ** 2))
    psnr = {"db": round(10 * np.log10(1.0 / max(mse, 1e-12)), 2), "max_abs": round(float(err.max()), 5),
            "frac_within_2_255": round(float(np.mean(err.max(axis=-1) <= 2.0 / 255.0)), 5), "res": [w, h],
            "against": "CPU oracle (line-by-line restatement of the reference path, oracle/), same inputs and RNG states; final sRGB RGB in [0,1]"}
    sample = {"frames_per_s": round(frac / dt, 5), "threads": O.lib().orc_num_threads(), "seconds": round(dt, 3),
              "what": f"one oracle Engine::frame of {config} at {w}x{h} ({frac:.3g} of the pixels), extrapolated by pixel count to "
                      f"{full['width']}x{full['height']}"}
    return sample, psnr


def latest_profile(prefix, config):
    """profiles/<prefix>_<round>_<config>.json of the newest round that has one (this round's first)."""
    for rnd in (ROUND, "r05", "r04", "r03", "r02", "r01"):
        path = os.path.join(REPO, "profiles", f"{prefix}_{rnd}_{config}.json")
        if os.path.exists(path):
            return path
    return None


def traffic_profile(config, samples_per_launch):
    """HBM bytes per launch of the roofline kernels from the newest PMC passes for this config
    (tools/gpu.sh pmc: separate FETCH_SIZE / WRITE_SIZE passes, gfx950 x2 FETCH correction), labelled
    with the file they came from.  The counted run must have launched the network on the same work as this
    line: a file whose samples per launch differ by more than 5 % (or that does not record them) is refused,
    and the reason is returned instead of the bytes.  None when no profile of this config exists."""
    path = latest_profile("pmc_traffic", config)
    if not path:
        return None
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    rel = os.path.relpath(path, REPO)
    spl = (d.get("roofline_kernels", {}).get("nerf_network_kernel") or {}).get("samples_per_launch")
    if not spl:
        return {"file": rel, "refused": "the file does not record the counted run's samples per network launch"}
    if abs(spl - samples_per_launch) > 0.05 * max(1.0, samples_per_launch):
        return {"file": rel, "refused": f"counted run: {spl:.0f} samples per launch, this line: {samples_per_launch:.0f} (> 5 % apart)"}
    return {"file": rel, "config": d.get("config"), "kernels": d.get("roofline_kernels", {}), "samples_per_launch": spl}


def valu_profile(config):
    """VALU roofline of the traversal kernels (tools/gpu.sh sq: SQ_INSTS_VALU per launch over the launch's duration
    in the same serialised counter pass; peak 1.229e12 wave64 VALU instructions/s), labelled with its file."""
    path = latest_profile("sq", config)
    if not path:
        return None
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    ks = d.get("kernels", {})
    out = {"source": os.path.relpath(path, REPO), "peak_wave_instr_per_s": 1.2288e12, "bound": "valu"}
    for k in ("raytrace_kernel", "shadow_rays_kernel"):
        if k in ks:
            v = ks[k]
            out[k] = {"valu_instr_per_launch": v.get("sq_insts_valu_per_launch"), "ms": round(v.get("avg_launch_ms", 0.0), 4),
                      "frac": round(v.get("valu_frac", 0.0), 4)}
    return out


def per_launch_table(stats):
    """Per launch index of a frame (the head round's network launch, the second round's, ...): the samples the
    launch evaluated (read by the kernel itself) and its duration (its own dispatch's HIP events), averaged over
    the frames; the line's `frac` is their sample-weighted figure (sum of bytes over sum of durations)."""
    out = []
    for k in range(max((len(s.network_launch) for s in stats), default=0)):
        rows = [s.network_launch[k] for s in stats if len(s.network_launch) > k]
        smp = sum(r[0] for r in rows) / len(rows)
        ms = sum(r[1] for r in rows) / len(rows)
        out.append({"index": k, "frames": len(rows), "samples": round(smp, 1), "ms": round(ms, 5),
                    "frac": round(smp * BYTES_PER_SAMPLE / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if ms > 0 else None})
    return out


def frame_cells(eng, cells, frames, warmup, px):
    """Render `frames` timed frames (after `warmup`) per parameter cell; frames/s (host wall clock around the
    synchronous sng_render_frame calls), samples per NeRF pixel and the network launches' roofline fraction."""
    import torch
    out = []
    for cell in cells:
        for k, v in cell.items():
            eng.set_param(k, v)
        warm_launches = 0
        for _ in range(warmup):
            warm_launches += int(eng.frame(spp=0, reset=True).network_launches)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = [eng.frame(spp=0, reset=True, collect_kernel_times=True) for _ in range(frames)]
        el = time.perf_counter() - t0
        net_ms = sum(r.ms_network for r in st)
        net_samples = sum(r.n_samples_network for r in st)
        gbs = net_samples * BYTES_PER_SAMPLE / (net_ms * 1e-3) / 1e9 if net_ms > 0 else 0.0
        ev = sum(r.n_samples - r.n_samples_reused for r in st)
        f_ms = sum(r.ms_network + r.ms_fused_tail + r.ms_onestep for r in st)
        fsw = ev * BYTES_PER_SAMPLE / (f_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if f_ms > 0 else 0.0
        r = st[-1]
        out.append({**cell, "frames_per_s": round(frames / el, 2), "ms_frame_device": round(r.ms_frame, 3),
                    "samples_per_px": round(r.n_samples / px, 3), "reference_slots_per_px": round(r.n_reference_slots / px, 3),
                    "hit_frac": round(r.n_hit / px, 4),
                    "network_roofline_frac": round(gbs / HBM_PEAK_GBS, 4), "field_sample_weighted_frac": round(fsw, 4),
                    "network_per_launch": per_launch_table(st),
                    "network_launches": {"warmup": warm_launches, "timed": int(sum(x.network_launches for x in st))},
                    "stages_ms": {"raytrace": round(r.ms_raytrace, 3), "nerf": round(r.ms_nerf, 3), "shadow": round(r.ms_shadow, 3)}})
    return out


def abm_sweep(model, frames, warmup):
    """The reference's own perf sweep (scripts/render/profiling.sh:12-18; every number in BASELINE.md): the lego
    snapshot + dmrf-compare-abm.json (armadillo, bunny, monkey, 2 lights) at 1280x720, --sshadows x --nshadows
    in {1,2,4,8}^2 (Engine::set_syn_samples / set_nerf_samples)."""
    from synerfgine_amd import scene as S
    tb, eng, _ = S.make_engine("abm", model=model)
    try:
        NW, NH = eng.resolution()["nerf"]
        cells = [{"sshadows": a, "nshadows": b} for a in (1, 2, 4, 8) for b in (1, 2, 4, 8)]
        return {"scene": "scenes/dmrf-compare-abm.json (scripts/virtual_desc/dmrf-compare-abm.json)", "model": model,
                "width": 1280, "height": 720, "frames_per_cell": frames,
                "cells": frame_cells(eng, cells, frames, warmup, NW * NH)}
    finally:
        tb.close()


def train_leg(steps=200, warmup=50, seed=1337, engine_params=None):
    """BASELINE config C5: online training on the reference's lego set (data/nerf/lego400, 95
    views, every 20th held out as tools/train_lego.py does) from a fresh init, batch 2^18 samples per step
    (m_training_batch_size, testbed.h:1103): `warmup` untimed steps, then `steps` timed ones (host wall clock
    around sng_train; the batch counters of NerfCounters::update_after_training, testbed_nerf.cu:3272-3296, are
    updated on the device, so the host does not wait for each step as the reference does -- DESIGN.md §7).  fp16 parameters / activations / gradient GEMM operands with f32 master
    weights and accumulation, tcnn's types (BASELINE.json C5 names bf16)."""
    import numpy as np
    from synerfgine_amd import Engine, Testbed, nerf_data, synthetic
    d = os.path.join(REPO, "data", "nerf", "lego400")
    imgs, xf, focal, pp = nerf_data.load_nerf_synthetic(d)
    angle = json.load(open(os.path.join(d, "transforms.json")))["camera_angle_x"]
    import math
    focal[:] = 0.5 * imgs.shape[2] / math.tan(0.5 * angle)   # the Blender focal
    train = [i for i in range(len(imgs)) if i % 20]
    tb = Testbed(0)
    try:
        cfg, params = synthetic.random_init(seed)
        tb.set_nerf_model(cfg, params)
        tb.set_training_dataset(imgs[train], xf[train], focal[train], pp[train])
        if engine_params:
            eng0 = Engine(tb)
            for k, v in engine_params.items():
                eng0.set_param(k, v)
        tb.train_reset(seed)
        tb.train(warmup)   # sng_train returns after its stream has finished (one host sync per step)
        t0 = time.perf_counter()
        st = tb.train(steps)
        el = time.perf_counter() - t0
        samples = int(st["measured_batch"])
        # algorithmic work of one step at the measured (compacted) batch: the five weight gradients dW = delta act^T
        # (K = samples; 64x32 + 16x64 + 64x32 + 64x64 + 16x64 = 10,240 weights), forward + backward of the fused MLPs,
        # and the hash-grid gradient scatter (8 levels x 8 corners x F = 4 f32 adds per sample)
        dw_flop = 2 * samples * 10240
        # per-stage device times of 50 more steps (HIP events per stage, param train_kernel_times; after the timed steps)
        # -> the roofline of each stage at its own bound
        eng = Engine(tb)
        eng.set_param("train_kernel_times", 1)
        st2 = tb.train(50)
        eng.set_param("train_kernel_times", 0)
        sm = st2.get("stage_ms", {})
        gb = 2 if eng.get_param("train_grid_grad_f16") else 4   # bytes per scattered gradient feature
        n_before = int(st2["measured_batch_before_compaction"])
        n_after = int(st2["measured_batch"])
        n_params = int(synthetic.n_params())
        rl = {}
        if sm:
            def frac(b, ms, peak):
                return round(b / (ms * 1e-3) / 1e9 / peak, 4) if ms > 0 else None
            rl = {"stage_ms": sm,
                  "network": {"bound": "hbm", "bytes": n_before * BYTES_PER_SAMPLE, "frac": frac(n_before * BYTES_PER_SAMPLE, sm["network"], HBM_PEAK_GBS),
                              "note": "inference forward of every generated sample, 548 B/sample (SURVEY 8d)"},
                  "field": {"bound": "float atomics", "bytes": n_after * 8 * 8 * 4 * gb, "peak_GBps": 1300.0,
                            "frac": frac(n_after * 8 * 8 * 4 * gb, sm["field"], 1300.0),
                            "note": f"hash-grid gradient scatter, 8 levels x 8 corners x 4 features x {gb} B per compacted sample "
                                    f"({'fp16 packed atomics, tcnn grad_t' if gb == 2 else 'f32 atomics'}), against the chip-wide float-atomic "
                                    "rate (MI355X_MICROARCH.md, Global float atomics, measured at the same byte rate for f32 and packed 16-bit "
                                    "adds); the kernel also runs the MLP forward + backward on MFMA and folds runs of equal entries before adding"},
                  "dw": {"bound": "hbm", "bytes": n_after * 960, "frac": frac(n_after * 960, sm["dw"], HBM_PEAK_GBS),
                         "mfma_tflops": round(dw_flop / (sm["dw"] * 1e-3) / 1e12, 2) if sm["dw"] > 0 else None,
                         "mfma_frac": round(dw_flop / (sm["dw"] * 1e-3) / 1e12 / MFMA_F16_PEAK_TFLOPS, 4) if sm["dw"] > 0 else None,
                         "note": "dW = delta act^T over K = samples: reads the 960 B/sample fp16 activation + gradient tiles once"},
                  "optimizer": {"bound": "hbm", "bytes_min": n_params * 20, "frac_min": frac(n_params * 20, sm["optimizer"], HBM_PEAK_GBS),
                                "note": "Ema(ExpDecay(Adam)) over every param: >= 20 B/param (gradient, master, EMA read; EMA, fp16 training "
                                        "and inference copies written) + 28 B per touched param (moments, step count)"},
                  "generate": {"bound": "latency", "rays": int(st2["rays_per_batch"]),
                               "note": "one march per training ray, 8 lanes per ray speculating 8 steps at a time (train_generate_spec_kernel); the samples then written in the batch slot the ray reserved"}}
        return {"steps_per_s": round(steps / el, 1), "ms_per_step": round(1e3 * el / steps, 3),
                "ms_per_step_device": round(st["ms"] / steps, 3), "steps": steps, "warmup": warmup,
                "batch_target": 1 << 18, "measured_batch": samples, "rays_per_batch": int(st["rays_per_batch"]),
                "loss_after": round(float(st["loss"]), 6), "step_after": int(st["step"]),
                "algorithmic_per_step": {"dw_gemm_flop": dw_flop, "mlp_fwd_bwd_flop": 3 * 20480 * samples,
                                         "grid_scatter_atomic_bytes": samples * 8 * 8 * 4 * 2},
                "roofline": rl,
                "dtype": "fp16 params / activations / GEMM operands / hash-grid gradients (tcnn's grad_t), f32 master weights, MLP gradients and accumulation "
                         "(tcnn's network_precision_t; BASELINE.json C5 says bf16)",
                "data": "data/nerf/lego400 (the reference's lego set at 400x400), 90 training views, fresh init (seed 1337)",
                "kernel_profile": f"profiles/{ROUND}_train_kernel_table.txt (rocprofv3 of tools/train_bench.py, this build)"}
    finally:
        tb.close()


def _srgb(rgba):
    import numpy as np
    lin = np.clip(rgba[..., :3], 0, None)
    return np.clip(np.where(lin < 0.0031308, 12.92 * lin, 1.055 * np.power(lin, 0.41666) - 0.055), 0, 1)


def orbit_leg(config, w, h, model, warmup, n=60):
    """The camera orbits the lego 1 degree per frame: nerf_spec_hint on vs off (alternating passes, mean of two each).
    The hints are read only when a frame repeats the previous frame's view (spec_view_key, host_render.cpp), so on the
    orbit both settings march with the opacity policy; the leg shows that hints cost nothing under motion."""
    import math

    import numpy as np
    import torch
    from synerfgine_amd import scene as S
    tb, eng, _ = S.make_engine(config, width=w, height=h, model=model)
    try:
        mats = []
        for k in range(n):
            ang = math.radians(1.0 * k)
            v = (0.62 * math.cos(ang) + 0.64 * math.sin(ang), 0.46, -0.64 * math.cos(ang) + 0.62 * math.sin(ang))
            tb.set_camera_view(v, (0.5, 0.5, 0.5), 1.0)
            mats.append(np.array(tb.camera_matrix))
        runs = {1: [], 0: []}
        for hint in (1, 0, 1, 0):
            eng.set_param("nerf_spec_hint", hint)
            for m in mats[:warmup]:
                tb.camera_matrix = m
                eng.frame(spp=0, reset=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for m in mats[warmup:]:
                tb.camera_matrix = m
                eng.frame(spp=0, reset=True)
            torch.cuda.synchronize()
            runs[hint].append((len(mats) - warmup) / (time.perf_counter() - t0))
        eng.set_param("nerf_spec_hint", 1)
        return {"frames_per_s": {"hints": round(sum(runs[1]) / 2, 1), "no_hints": round(sum(runs[0]) / 2, 1)},
                "passes": {"hints": [round(x, 1) for x in runs[1]], "no_hints": [round(x, 1) for x in runs[0]]},
                "res": [w, h], "config": config,
                "note": "camera orbiting the lego 1 degree per frame; hints are read only for a repeated view (spec_view_key)"}
    finally:
        tb.close()


def c4fox_leg(frames=10, warmup=2, config="c4fox"):
    """C4's workload on a trained cascaded field (config c4fox: the reference's fox capture trained by tools/train_fox.py,
    scenes/fox-rocks.json) at 1920x1080: frames/s, the network launches' per-launch roofline, and the march schedule of
    the frame (trace_alt's one-step regime length, multi-step rounds, how many rays are still alive at the regime's end and
    near MARCH_ITER) from the per-iteration march log; then which of C4's exact schedule optimisations pay on this field:
    the same frames with the ray-local one-step regime off (nerf_onestep 0: the regime's iterations as whole-GPU launches)
    and with the multi-step speculative rounds off (nerf_msr 0)."""
    import numpy as np
    import torch
    from synerfgine_amd import scene as S
    if not os.path.exists(S.FOX_INGP):
        return {"error": "data/fox.ingp not present"}
    tb, eng, _ = S.make_engine(config, model="fox")
    try:
        res = eng.resolution()
        NW, NH = res["nerf"]
        px = NW * NH
        variants = [{}, {"nerf_onestep": 0}, {"nerf_onestep": 1, "nerf_msr": 0}, {"nerf_onestep": 1, "nerf_msr": 1}] if config == "c4fox" else [{}]
        cells = frame_cells(eng, variants, frames, warmup, px)
        base = cells[0]
        eng.set_param("march_log", 1)
        r = eng.frame(spp=0, reset=True)
        log = eng.frame_buffer("march_log", np.uint32).reshape(-1, 3)[: min(r.n_iterations, 2048)]
        eng.set_param("march_log", 0)
        alive = log[:, 0].astype(np.int64)
        os_end = r.onestep_from_iter + r.onestep_iterations
        out = {"workload": WORKLOADS[config], "snapshot": os.path.relpath(S.FOX_INGP, REPO), "res": [NW, NH],
               "frames_per_s": base["frames_per_s"], "ms_frame_device": base["ms_frame_device"], "samples_per_px": base["samples_per_px"],
               "reference_slots_per_px": base["reference_slots_per_px"], "hit_frac": base["hit_frac"],
               "network_roofline_frac": base["network_roofline_frac"], "network_per_launch": base["network_per_launch"],
               "stages_ms": base["stages_ms"],
               "schedule": {"iterations": int(r.n_iterations), "onestep_regime": [int(r.onestep_from_iter), int(r.onestep_iterations)],
                            "msr_rounds": int(r.msr_rounds), "alive_at_start": int(alive[0]) if len(alive) else 0,
                            "alive_after_onestep_regime": int(alive[os_end]) if os_end < len(alive) else 0,
                            "alive_frac_after_onestep_regime": round(float(alive[os_end]) / px, 5) if os_end < len(alive) else 0.0,
                            "rays_reaching_march_iter": int(alive[-1]) if r.n_iterations >= 10000 else 0,
                            "note": "alive = rays of the iteration (per-iteration march log); a ray still alive at MARCH_ITER (10000) "
                                    "is a nearly transparent one, the kind that makes 97 % of the synthetic C4 frame's work"}}
        if config == "c4fox":
            out["optimisations"] = {"onestep_regime_off": {k: cells[1][k] for k in ("frames_per_s", "ms_frame_device", "network_roofline_frac")},
                                    "msr_rounds_off": {k: cells[2][k] for k in ("frames_per_s", "ms_frame_device", "network_roofline_frac")},
                                    "default_again": {k: cells[3][k] for k in ("frames_per_s", "ms_frame_device")}}
        return out
    finally:
        tb.close()


def nerf_views(model, frames, warmup, cpu_check=True):
    """NeRF-dominated legs (no virtual objects): (a) BASELINE config C2 -- 800x800 at the lego dataset's camera 0
    (transforms.json frame 0, nerf_matrix_to_ngp, its camera_angle_x field of view; a view train_lego.py held
    out), with the model's PSNR against that dataset image (ngp render, 400x400) and the frame's PSNR against the
    CPU oracle (200x200); (b) a 1920x1080 close-up: of three zooms with the camera outside the unit cube, the one
    whose rays hit the object most."""
    import math

    import numpy as np
    from synerfgine_amd import nerf_data
    from synerfgine_amd import scene as S
    d = os.path.join(REPO, "data", "nerf", "lego400")
    meta = json.load(open(os.path.join(d, "transforms.json")))
    fr0 = meta["frames"][0]
    cam = nerf_data.nerf_matrix_to_ngp(fr0["transform_matrix"])          # [3 rows, 4 cols]
    w0 = int(meta.get("w", 400))
    # the focal data/lego.ingp was trained with (tools/train_lego.py FOCAL_FROM_ANGLE=1): the Blender
    # camera_angle_x, not the fl_x the file also carries
    fov = math.degrees(meta["camera_angle_x"])
    out = {"model": model}
    tb, eng, (ncfg, params, grid) = S.make_engine("c2", width=800, height=800, model=model)
    try:
        tb.camera_matrix = np.asarray(cam, np.float32).T.reshape(-1)
        tb.set_fov(fov)
        NW, NH = eng.resolution()["nerf"]
        leg = frame_cells(eng, [{}], frames, warmup, NW * NH)[0]
        leg.update({"res": [NW, NH], "camera": "data/nerf/lego400/transforms.json frames[0] (" + fr0["file_path"] + "), fov %.3f deg" % fov})
        # model quality at the dataset's resolution: ngp render path (render_mode Shade) vs the image, premultiplied on black
        eng.init(w0, w0)
        tb.camera_matrix = np.asarray(cam, np.float32).T.reshape(-1)
        tb.set_fov(fov)
        rgba = eng.render_nerf(render_mode=1).download("nerf_rgba")
        gt = nerf_data.read_png(os.path.join(d, fr0["file_path"].lstrip("./") + ("" if fr0["file_path"].endswith(".png") else ".png"))).astype(np.float32) / 255.0
        mse = float(np.mean((_srgb(rgba) - gt[..., :3] * gt[..., 3:4]) ** 2))
        leg["psnr_vs_dataset_image_db"] = round(10 * np.log10(1.0 / max(mse, 1e-12)), 2)
        if cpu_check:
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import oracle as O
            eng.init(200, 200)
            tb.camera_matrix = np.asarray(cam, np.float32).T.reshape(-1)
            tb.set_fov(fov)
            nrng, mrng = eng.rng_states(0).copy(), eng.rng_states(1).copy()
            got = eng.frame(spp=0, reset=True).download("final_rgba")
            ref = O.render_frame(O.Model(ncfg, params), O.volume_for(ncfg, grid), tb, eng, nrng, mrng)["final"]
            err = np.abs(np.clip(got[..., :3], 0, 1) - np.clip(ref[..., :3], 0, 1))
            leg["psnr_vs_oracle_db"] = round(10 * np.log10(1.0 / max(float(np.mean(err ** 2)), 1e-12)), 2)
            leg["psnr_vs_oracle_res"] = [200, 200]
        out["c2_dataset_view"] = leg
    finally:
        tb.close()
    # (c) a moving camera: an orbit of 1 degree per frame at C2 (800x800) and at the benchmarked C3 (1080p + mesh)
    out["c2_orbit_1deg_per_frame"] = orbit_leg("c2", 800, 800, model, warmup)
    out["c3_orbit_1deg_per_frame"] = orbit_leg("c3", 1920, 1080, model, warmup)
    tb, eng, _ = S.make_engine("c2", width=1920, height=1080, model=model)
    try:
        NW, NH = eng.resolution()["nerf"]
        pick = None
        for scale in (1.2, 1.0, 0.9):   # camera distance from the centre >= 0.9 > the cube's half diagonal
            tb.set_camera_view((0.62, 0.46, -0.64), (0.5, 0.5, 0.5), scale)
            r = eng.frame(spp=0, reset=True)
            hf = r.n_hit / float(NW * NH)
            if pick is None or hf > pick[1]:
                pick = (scale, hf)
        tb.set_camera_view((0.62, 0.46, -0.64), (0.5, 0.5, 0.5), pick[0])
        leg = frame_cells(eng, [{}], frames, warmup, NW * NH)[0]
        leg.update({"res": [NW, NH], "camera": "view dir (0.62, 0.46, -0.64) at (0.5, 0.5, 0.5), zoom scale %.2f" % pick[0]})
        out["frame_filling_1080p"] = leg
    finally:
        tb.close()
    return out


def bvh_leg(eng, config, s0):
    """BVH work of one C3/C4 frame: a lane-level counting frame (rt_count = 1: world queries, box and triangle tests) and a
    wave-level one (rt_count = 2: wave iterations of the record and triangle loops), both rendered by the counting
    instantiations of the traversal kernels (bit-identical frames, untimed).  lane_eff = lane work / (64 x wave
    iterations); useful_frac = the kernel's VALU issue fraction (profiles/sq_*.json) x the record loop's lane_eff."""
    cnt = {}
    for mode in (1, 2):
        eng.set_param("rt_count", mode)
        eng.frame(spp=0, reset=True)
        cnt[mode] = eng.rt_counters()
    eng.set_param("rt_count", 0)
    lane, wave = cnt[1], cnt[2]
    eff = {k: {"record_loop": round(lane[k]["box_tests"] / 2 / max(1, 64 * wave[k]["box_tests"]), 4),
               "tri_loop": round(lane[k]["tri_tests"] / max(1, 64 * wave[k]["tri_tests"]), 4)} for k in ("path", "shadow")}
    valu = valu_profile(config)
    useful, algo = {}, {}
    if valu:
        for kern, k in (("raytrace_kernel", "path"), ("shadow_rays_kernel", "shadow")):
            if kern in valu:
                useful[kern] = round(valu[kern]["frac"] * eff[k]["record_loop"], 4)
                # the tests' own arithmetic over the serialized launch duration of the same SQ pass, at the FP32 vector peak
                ms = valu[kern]["ms"]
                ops = lane[k]["box_tests"] * BOX_TEST_OPS + lane[k]["tri_tests"] * TRI_TEST_OPS
                algo[kern] = round(ops / (ms * 1e-3) / (FP32_VECTOR_PEAK_TFLOPS * 1e12), 4) if ms else None
    rt_s = s0.ms_raytrace * 1e-3
    q = lane["path"]["queries"] + lane["shadow"]["queries"]
    return {"per_frame": lane, "lane_eff": eff, "valu_roofline": valu, "useful_frac": useful, "algorithmic_flop_frac": algo,
            "flops_per_test": {"box": BOX_TEST_OPS, "triangle": TRI_TEST_OPS, "peak_tflops": FP32_VECTOR_PEAK_TFLOPS},
            "rays_per_s": round(q / rt_s, 1) if rt_s > 0 else None, "raytrace_stage_ms": round(s0.ms_raytrace, 3)}


def extra_legs(eng, res, args):
    """The legs behind --extras: C3 with NeRF shadows r = 1/4, the reference's own dmrf-compare-abm sweep, the
    NeRF-dominated views and orbits, and C4's workload on the trained fox field."""
    from synerfgine_amd import scene as S
    out = {}
    try:
        if args.config == "c3":
            NW, NH = res["nerf"]
            out["c3_nerf_shadow_r"] = frame_cells(eng, [{"nerf_shadow_samples": 1}, {"nerf_shadow_samples": 4}], 5, 1, NW * NH)
            eng.set_param("nerf_shadow_samples", 1)
    except Exception as e:
        out["c3_nerf_shadow_r"] = {"error": repr(e)}
    try:
        out["abm_sweep"] = abm_sweep(args.model if args.config not in ("c4", "c4fox", "foxarm") else "lego", 3, 1)
    except Exception as e:
        out["abm_sweep"] = {"error": repr(e)}
    try:
        if os.path.exists(S.LEGO_INGP):
            out["nerf_views"] = nerf_views("lego", 10, 2, cpu_check=not args.no_cpu_baseline)
    except Exception as e:
        out["nerf_views"] = {"error": repr(e)}
    for cfg in ("c4fox", "foxarm"):
        try:
            if args.config != cfg:
                out[cfg] = c4fox_leg(config=cfg)
        except Exception as e:
            out[cfg] = {"error": repr(e)}
    return out


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def compact_line(full):
    """The one stdout line: the driver contract's keys, `config`, `roofline` (frac, per-launch rows, the uncontended
    figure, traffic), `cpu_baseline`, `psnr_vs_oracle` and summaries of the BVH and training legs.  Everything else
    (the extra legs, notes, per-run lists) goes to --extras' file; the line names the committed one of this build.
    Kept under LINE_MAX_BYTES: optional parts are dropped, least important first, if it would be longer."""
    line = _pick(full, ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                        "vs_baseline", "dtype", "data"))
    line["config"] = _pick(full.get("config", {}), ("workload", "width", "height", "nerf_res", "tiles", "step_schedule",
                                                    "samples_per_frame", "hit_rays"))
    if "streams" in full:
        line["streams"] = full["streams"]
    if full.get("overrides"):
        line["overrides"] = full["overrides"]
    line["stages_ms_last_frame"] = full.get("stages_ms_last_frame")
    rf = full.get("roofline", {})
    r = _pick(rf, ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_source", "traffic_over_algorithmic",
                   "algorithmic_bytes_per_sample", "avg_launch_ms", "launches", "warmup_launches", "samples_in_launches", "per_launch",
                   "mfma_frac"))
    if "field_sample_weighted" in rf:
        r["field_sample_weighted"] = _pick(rf["field_sample_weighted"], ("frac",))
    if "onestep_regime" in rf:
        r["onestep_regime"] = _pick(rf["onestep_regime"], ("ms",))
    unc = rf.get("uncontended")
    if isinstance(unc, dict):
        r["uncontended"] = _pick(unc, ("frac", "source", "frames_per_s", "warmup_launches", "launches", "error"))
        alt = (unc.get("alternates") or {}).get("hip_events_this_process")
        if alt:
            r["uncontended"]["alternates"] = {"hip_events_this_process": _pick(alt, ("frac", "per_launch"))}
    line["roofline"] = r
    b = full.get("bvh")
    if isinstance(b, dict):
        v = b.get("valu_roofline") or {}
        line["bvh"] = {"lane_eff": b.get("lane_eff"), "useful_frac": b.get("useful_frac"),
                       "algorithmic_flop_frac": b.get("algorithmic_flop_frac"), "rays_per_s": b.get("rays_per_s"),
                       "valu_frac": {k: v[k]["frac"] for k in ("raytrace_kernel", "shadow_rays_kernel") if k in v},
                       "valu_source": v.get("source"), "error": b.get("error")}
        line["bvh"] = {k: x for k, x in line["bvh"].items() if x is not None}
    t = full.get("train")
    if isinstance(t, dict):
        rl = t.get("roofline") or {}
        line["train"] = {**_pick(t, ("steps_per_s", "ms_per_step", "measured_batch", "loss_after", "kernel_profile", "error")),
                         "stage_ms": rl.get("stage_ms"),
                         "frac": {k: rl[k].get("frac", rl[k].get("frac_min")) for k in ("network", "field", "dw", "optimizer") if k in rl}}
    cb = full.get("cpu_baseline")
    if isinstance(cb, dict):
        c = _pick(cb, ("value", "unit", "cores", "kind", "sample", "cpu_model", "cgroup_cpu_quota", "error"))
        legs = cb.get("legs") or {}
        if "one_thread" in legs:
            c["one_thread_frames_per_s"] = legs["one_thread"]["frames_per_s"]
        ws = cb.get("benchmarked_workload_sample")
        if ws:
            c["benchmarked_workload_sample"] = _pick(ws, ("frames_per_s", "threads", "seconds"))
        line["cpu_baseline"] = c
    if "psnr_vs_oracle" in full:
        line["psnr_vs_oracle"] = _pick(full["psnr_vs_oracle"], ("db", "max_abs", "frac_within_2_255", "res", "error"))
    line["extras"] = EXTRAS_FILE
    for drop in (("roofline", "uncontended", "alternates"), ("roofline", "traffic_source"), ("bvh",), ("train", "stage_ms"),
                 ("stages_ms_last_frame",), ("roofline", "per_launch"), ("data",), ("config", "tiles")):
        if len(json.dumps(line)) <= LINE_MAX_BYTES:
            break
        d = line
        for k in drop[:-1]:
            d = d.get(k, {}) if isinstance(d, dict) else {}
        if isinstance(d, dict):
            d.pop(drop[-1], None)
    return line


def emit_line(line):
    """Rank 0's one JSON line, last on stdout (stderr flushed first so nothing interleaves with it)."""
    sys.stderr.flush()
    sys.stdout.write(json.dumps(line) + "\n")
    sys.stdout.flush()


def frame_result(args, stats, elapsed, world, res, bounds, comm, overrides, root_gather, on_dev, model_data):
    """The full result of the timed frames (rank 0): the driver contract's keys, config, and the roofline of the
    dominant kernel from the frames' own per-launch HIP events and sample counters.  `stats` are sng_frame_result
    mirrors (attributes only), so the CPU tests build this from stub frames."""
    # dominant kernel: fused hash-grid + MLP, timed with hipEvents on its own stream over the timed region.
    # Samples per launch come from the device counter of the network launches (MarchCtrl::net_samples);
    # the ray-local fused tail (fused.hip) evaluates the rest of the frame's samples inside its own kernel.
    ms_net = sum(s.ms_network for s in stats)
    launches = sum(s.network_launches for s in stats)
    samples = sum(s.n_samples_network for s in stats)
    total_samples = sum(s.n_samples for s in stats)          # march samples composited
    reused = sum(s.n_samples_reused for s in stats)         # of which taken from the boundary-sample cache
    evaluated = total_samples - reused                      # network evaluations (launches + fused tail)
    spec_evals = sum(s.spec_evals for s in stats)           # speculative tail rounds: samples their network launches evaluated
    spec_exec = sum(s.spec_exec for s in stats)             # ... of which composited (the rest: look-ahead past a ray's end)
    msr_evals = sum(s.msr_evals for s in stats)             # multi-step speculative rounds: samples their launches evaluated
    msr_exec = sum(s.msr_exec for s in stats)               # ... of which the per-iteration wavefront would have evaluated
    tail_samples = evaluated - (samples - (spec_evals - spec_exec) - (msr_evals - msr_exec))
    ms_tail = sum(s.ms_fused_tail for s in stats)
    os_evals = sum(s.onestep_field_evals for s in stats)   # field evaluations inside the one-step regime's final pass
    ms_os = sum(s.ms_onestep for s in stats)
    tail_samples -= os_evals
    avg_launch_ms = ms_net / max(1, launches)
    per_launch = per_launch_table(stats)
    bytes_per_launch = samples * BYTES_PER_SAMPLE / max(1, launches)
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
    tflops = samples * FLOPS_PER_SAMPLE / (ms_net * 1e-3) / 1e12 if ms_net > 0 else 0.0
    tail_gbs = tail_samples * BYTES_PER_SAMPLE / (ms_tail * 1e-3) / 1e9 if ms_tail > 0 else 0.0
    field_ms = ms_net + ms_tail
    field_gbs = evaluated * BYTES_PER_SAMPLE / (field_ms * 1e-3) / 1e9 if field_ms > 0 else 0.0
    prof = traffic_profile(args.config, samples / max(1, launches))
    traffic = None
    if prof and "refused" not in prof:
        net_prof = prof["kernels"].get("nerf_network_kernel")
        traffic = net_prof.get("hbm_bytes_per_launch") if net_prof else None

    fps = args.steps / elapsed
    s0 = stats[-1]
    result = {
        "metric": METRICS[args.config],
        "value": round(fps, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp16 (hash grid + MLP, MFMA f16->f32), fp32 (marching, compositing, shading)",
        "data": (f"snapshot {model_data}" +
                 (" (base.json NeRF L=8,F=4,T=2^19 trained on-GPU by tools/train_lego.py from the reference's lego set, data/nerf/lego400)"
                  if args.model == "lego" else "") if args.model != "synthetic" else
                 "synthetic: random-init base.json NeRF (L=8,F=4,T=2^19) with an analytic density (synthetic.py)") +
                "; scene JSON + OBJ meshes from scenes/ and data/obj/; synthetic frames (fixed camera, accumulation reset every frame)",
        "config": {"workload": f"{args.config}: " + WORKLOADS[args.config],
                   "width": res["mesh"][0], "height": res["mesh"][1], "nerf_res": list(res["nerf"]),
                   "tiles": f"{world} horizontal bands (rows {bounds}) + " +
                            (("RCCL gather of the RGBA8 bands to rank 0 (sng_gather_rgba8)" if root_gather else
                              "RCCL all_gather of RGBA8 tiles" if on_dev else "gloo gather of the RGBA8 bands to rank 0 (tiling.gather_to_root)")
                             if world > 1 else "no gather"),
                   "step_schedule": "band-local" if (world > 1 and args.local_schedule) else ("frame-wide (per-iteration alive-count all-reduce)" if world > 1 else "frame-wide"),
                   "samples_per_frame": int(s0.n_samples), "samples_reused_per_frame": int(s0.n_samples_reused),
                   "reference_slots_per_frame": int(s0.n_reference_slots),
                   "wavefront_iterations": int(s0.n_iterations), "fused_tail_from_iteration": int(s0.fused_from_iter),
                   "onestep_regime": [int(s0.onestep_from_iter), int(s0.onestep_iterations)],
                   "hit_rays": int(s0.n_hit)},
        "comm": comm,
        "streams": "serialized (raytracer then NeRF)" if args.serial_streams else
                   "concurrent (NeRF head alone, then raytracer || NeRF tail; NeRF stream high priority)",
        "overrides": overrides,
        "stages_ms_last_frame": {"frame": round(s0.ms_frame, 3), "raytrace": round(s0.ms_raytrace, 3), "nerf": round(s0.ms_nerf, 3),
                                 "shadow": round(s0.ms_shadow, 3), "overlay": round(s0.ms_overlay, 3)},
        "temporal_hints": "the speculative NeRF tail sizes each ray's look-ahead by its pixel's ray life in the previous "
                          "frame (nerf_spec_hint; exact whatever the hint), read only when the frame repeats that frame's view "
                          "(spec_view_key); the timed frames repeat one camera, so after the first frame the hints are read; "
                          "nerf_views.c2_orbit_1deg_per_frame / c3_orbit_1deg_per_frame measure a moving camera",
        "roofline": {"kernel": "nerf_network_kernel<4,1> (fused hash grid + SH + density/rgb MLP)", "bound": "hbm",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": prof["file"] if prof else None,
                     "traffic_refused": prof.get("refused") if prof else None,
                     "traffic_over_algorithmic": round(traffic / bytes_per_launch, 4) if traffic and bytes_per_launch else None,
                     "algorithmic_bytes_per_sample": BYTES_PER_SAMPLE,
                     "avg_launch_ms": round(avg_launch_ms, 5), "launches": launches, "samples_in_launches": int(samples),
                     "per_launch": per_launch,
                     "timing": "HIP events recorded by each launch's own dispatch (hipExtLaunchKernelGGL start/stop events) on the NeRF stream over the timed region" +
                               ("" if args.serial_streams else "; the kernel shares the GPU with the raytracer stream, so this is the "
                                "contended duration (uncontended: --serial-streams)"),
                     "mfma_tflops": round(tflops, 2), "mfma_frac": round(tflops / MFMA_F16_PEAK_TFLOPS, 4),
                     "fused_tail": {"kernel": "nerf_fused_kernel (march + field + composite, ray-local)", "samples": int(tail_samples),
                                    "ms": round(ms_tail, 4), "achieved": round(tail_gbs, 1), "frac": round(tail_gbs / HBM_PEAK_GBS, 4),
                                    "timing": "hipEvents around the tail launch (it runs beside the raytracer on reserved CUs in the "
                                              "concurrent schedule, so its duration is latency, not throughput)"},
                     "spec_tail": {"kernels": "spec_generate (K iterations marched ahead per ray) + nerf_network_kernel + spec_composite "
                                              "(exact replay), per round", "rounds_per_frame": int(s0.spec_rounds),
                                   "samples_evaluated": int(spec_evals), "samples_composited": int(spec_exec),
                                   "lookahead_discarded_frac": round(1.0 - spec_exec / spec_evals, 4) if spec_evals else 0.0},
                     "msr_rounds": {"kernels": "msr_generate (K iterations of S steps marched ahead per ray) + nerf_network_kernel + "
                                               "msr_count (death histogram) + msr_schedule (committed prefix) + msr_commit (exact replay), "
                                               "while n_steps is 2..7", "rounds_per_frame": int(s0.msr_rounds),
                                    "samples_evaluated": int(msr_evals), "samples_committed": int(msr_exec),
                                    "discarded_frac": round(1.0 - msr_exec / msr_evals, 4) if msr_evals else 0.0},
                     "onestep_regime": {"kernels": "nerf_onestep_kernel x2 + schedule (trace_alt while n_alive > target/2; ray-local, "
                                                   "periodic rays composited in a closed loop)", "field_evals": int(os_evals),
                                        "ms": round(ms_os, 4)},
                     "field_sample_weighted": {"samples": int(evaluated), "ms": round(field_ms + ms_os, 4),
                                               "achieved": round(evaluated * BYTES_PER_SAMPLE / ((field_ms + ms_os) * 1e-3) / 1e9, 1) if field_ms + ms_os > 0 else 0.0,
                                               "frac": round(evaluated * BYTES_PER_SAMPLE / ((field_ms + ms_os) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if field_ms + ms_os > 0 else 0.0}},
    }
    return result


def dry_run(args, rank, world):
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([1], dtype=torch.int64)
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_formed": int(t.item()), "world_size": dist.get_world_size(),
                          "requested_gpus": args.gpus}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        return dry_run(args, rank, world)
    import numpy as np
    import torch
    import torch.distributed as dist

    n_dev = torch.cuda.device_count()
    dev_id = local_rank % max(1, n_dev)   # ranks > GPUs only in the gloo rehearsal mode (--dist-backend gloo)
    if world > 1:
        torch.cuda.set_device(dev_id)
        dist.init_process_group(args.dist_backend)
        assert dist.get_world_size() == args.gpus, "process group does not span --gpus ranks"
    from synerfgine_amd import scene as S
    from synerfgine_amd import tiling as T

    overrides = {"concurrent_streams": 0} if args.serial_streams else {}
    for kv in args.set:
        k, v = kv.split("=", 1)
        overrides[k] = float(v)
    if args.model is None:
        args.model = "fox" if args.config in ("c4fox", "foxarm") else "lego" if (args.config != "c4" and os.path.exists(S.LEGO_INGP)) else "synthetic"
    tb, eng, eng_cfg = S.make_engine(args.config, device_id=dev_id, overrides=overrides, model=args.model)
    res = eng.resolution()
    MW, MH = res["mesh"]
    dev = torch.device("cuda", dev_id)
    stream = torch.cuda.current_stream(dev)
    bounds = T.even_bounds(MH, world)
    comm = {"backend": args.dist_backend if world > 1 else None, "world_size": dist.get_world_size() if world > 1 else 1}
    if world > 1 and not args.local_schedule:
        # frame-wide step schedule: one uint32 all-reduce per wavefront iteration
        # keeps every band bit-identical to the single-GPU frame
        if args.dist_backend == "nccl":
            eng.attach_comm()
            comm["sched_comm"] = f"RCCL communicator of {world} ranks (sng_set_comm)"
        else:
            def _reduce(vals):
                t = torch.tensor(vals, dtype=torch.int64)
                dist.all_reduce(t)
                return t.tolist()
            eng.attach_host_reducer(_reduce)
            comm["sched_comm"] = f"gloo host reducer over {world} ranks"

    if world > 1 and not args.even_bands:
        # untimed calibration: re-split the rows until every band costs the same device time
        # (sky rows are ~free, object rows ~100x dearer), then keep the split fixed
        for _ in range(args.balance_iters):
            r = eng.frame(spp=0, reset=True, rows=(bounds[rank], bounds[rank + 1]))
            t = torch.tensor([r.ms_frame], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
            ts = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(ts, t)
            bounds = T.balance_bounds(MH, bounds, [float(x.item()) for x in ts])
    rows = (bounds[rank], bounds[rank + 1])
    band = max(bounds[k + 1] - bounds[k] for k in range(world))
    on_dev = args.dist_backend == "nccl"
    # composition: RGBA8 (4 B/px).  RCCL: every band goes to rank 0 only, received straight
    # into its rows of the frame (sng_gather_rgba8: grouped ncclSend / ncclRecv).  gloo (CPU rehearsal):
    # sng_final_rgba8 tiles all-gathered on the host.
    tile_dev = torch.zeros((band, MW), dtype=torch.int32, device=dev)
    tile = torch.zeros((band, MW), dtype=torch.int32)
    root_gather = world > 1 and on_dev and not args.local_schedule   # the communicator sng_set_comm attached
    if root_gather:
        frame = torch.empty((MH, MW), dtype=torch.int32, device=dev) if rank == 0 else None
    elif on_dev:
        frame = torch.empty((world * band, MW), dtype=torch.int32, device=dev) if world > 1 else None
    else:   # gloo: the bands reassembled into rank 0's frame by their bounds (tiling.gather_to_root)
        frame = torch.empty((MH, MW), dtype=torch.int32) if world > 1 and rank == 0 else None

    def step(collect):
        r = eng.frame(spp=0, reset=True, rows=rows if world > 1 else None, collect_kernel_times=collect)
        if root_gather:
            eng.gather_rgba8(bounds, frame.data_ptr() if rank == 0 else 0)
        elif world > 1:
            if rows[1] > rows[0]:
                tb._lib.sng_final_rgba8(tb.ctx, rows[0], rows[1], tile_dev.data_ptr(), stream.cuda_stream)
            if on_dev:
                T.gather_bands(tile_dev, frame)
            else:
                tile.copy_(tile_dev)
                T.gather_to_root(tile, bounds, frame)
        return r

    warm_launches = 0   # network launches of the warm-up frames (tools/roofline_check.py aligns the kernel trace on them)
    for _ in range(args.warmup):
        warm_launches += int(step(False).network_launches)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        stats.append(step(True))
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev if on_dev else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    result, s0 = None, stats[-1]
    if rank == 0:
        snap = S.snapshot_path(args.config, args.model)
        result = frame_result(args, stats, elapsed, world, res, bounds, comm, overrides, root_gather, on_dev,
                              os.path.relpath(snap, REPO) if snap else None)
        result["roofline"]["warmup_launches"] = warm_launches
    if rank == 0 and world == 1 and not args.no_sweep:
        # extra legs, after the timed region: the same workload with the two streams serialized (the roofline kernel's
        # launches then run alone), the BVH work of one counting frame, and the training step (config C5)
        if not args.serial_streams:
            try:
                NW, NH = res["nerf"]
                u = frame_cells(eng, [{"concurrent_streams": 0}], 10, 2, NW * NH)[0]
                eng.set_param("concurrent_streams", 1)
                chk = os.path.join(REPO, "profiles", f"{ROUND}_roofline_check.json")
                same = json.load(open(chk)).get("uncontended") if os.path.exists(chk) else None
                # one source per figure: the uncontended frac is the rocprofv3 trace's (the same bench.py command under
                # tools/gpu.sh profdriver, durations from the kernel trace); this process's HIP events are the labelled
                # alternate (a ~6 us launch's HIP-event duration is ~2x its trace duration)
                result["roofline"]["uncontended"] = {
                    "frac": round(same["rocprof_frac"], 4) if same and "rocprof_frac" in same else u["network_roofline_frac"],
                    "source": (f"rocprofv3 kernel trace of the driver-format command ({os.path.relpath(chk, REPO)}, tools/gpu.sh profdriver)"
                               if same and "rocprof_frac" in same else "HIP events of this process (no rocprof check of this round)"),
                    "alternates": {"hip_events_this_process": {"frac": u["network_roofline_frac"], "per_launch": u["network_per_launch"]}},
                    "warmup_launches": u["network_launches"]["warmup"], "launches": u["network_launches"]["timed"],
                    "field_sample_weighted_frac": u["field_sample_weighted_frac"],
                    "frames_per_s": u["frames_per_s"],
                    "note": "the same frames with the raytracer and the NeRF serialized (concurrent_streams=0, 10 frames after "
                            "the timed region): the network launches run alone"}
            except Exception as e:
                result["roofline"]["uncontended"] = {"error": repr(e)}
        try:
            if args.config in ("c3", "c4"):
                result["bvh"] = bvh_leg(eng, args.config, s0)
        except Exception as e:
            result["bvh"] = {"error": repr(e)}
        if args.extras:
            result.update(extra_legs(eng, res, args))
        try:
            result["train"] = train_leg()
        except Exception as e:
            result["train"] = {"error": repr(e)}
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        try:
            legs, threads = cpu_baseline_c1(args.model if args.config not in ("c4", "c4fox", "foxarm") else "lego", args.cpu_runs)
            best = legs[threads]
            result["cpu_baseline"] = {
                "value": best["frames_per_s"], "unit": "frames/s", "cores": threads, "kind": "port",
                "sample": "BASELINE config C1: the oracle (C++ OpenMP restatement of the render path; the reference has no CPU "
                          "path) renders the lego snapshot at 256x256, NeRF only; median of "
                          f"{args.cpu_runs} after 1 warm-up",
                "legs": {"all_threads": best, "one_thread": legs[1]}, **cpu_info()}
        except Exception as e:   # the CPU leg must never hide the GPU number
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
    tb.close()
    if rank == 0:
        if not args.no_cpu_baseline and world == 1:
            try:
                sample, result["psnr_vs_oracle"] = cpu_sample_c3(eng_cfg, args.config, args.cpu_baseline_scale, args.model, overrides)
                result["cpu_baseline"]["benchmarked_workload_sample"] = sample
            except Exception as e:
                result["psnr_vs_oracle"] = {"error": repr(e)}
        if args.extras:
            os.makedirs(os.path.dirname(os.path.abspath(args.extras)), exist_ok=True)
            with open(args.extras, "w") as f:
                json.dump(result, f, indent=1)
        emit_line(compact_line(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
