"""Multi-GPU band path: row bands rendered by separate ranks, with the frame-wide
step schedule exchanged every wavefront iteration, reproduce the single-GPU frame bit for bit.

The ranks here are processes sharing the one GPU of the test box; the schedule exchange runs
through the host reducer (gloo all_reduce), the transport-independent half of sng_set_comm.
The RCCL transport itself is checked at world size 1 (a second rank cannot share the GPU).
"""
import os
import socket
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
# a smaller wavefront budget than the default 2^21 so that clamp(target / n_alive, 1, 8) varies
# over the iterations (at 2^21 every C3 iteration takes 8 steps and the schedule is moot)
TARGET = 1 << 17


def _prefix_equal(a, b):
    n = min(len(a), len(b))   # the fused tail may end a band's iterations early
    return n > 0 and np.array_equal(a[:n], b[:n])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _band_worker(rank, world, port, bounds, overrides, out_dir, config="c3", target=TARGET):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from synerfgine_amd import scene as S
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tb, eng, _ = S.make_engine(config, overrides=overrides)

        def reduce_fn(vals):
            t = torch.tensor(vals, dtype=torch.int64)
            dist.all_reduce(t)
            return t.tolist()

        r0, r1 = bounds[rank], bounds[rank + 1]
        rng = [eng.rng_states(0), eng.rng_states(1)]

        def fresh():   # every frame below starts from the same per-pixel RNG streams
            eng.set_rng_states(0, rng[0])
            eng.set_rng_states(1, rng[1])

        res = {}
        # independent bands (local schedule) first, then the frame-wide schedule
        fresh()
        r = eng.frame(rows=(r0, r1), target_n_queries=target)
        res["local_steps"] = np.array(r.steps_per_iter, np.int64)
        eng.attach_host_reducer(reduce_fn)
        fresh()
        r = eng.frame(rows=(r0, r1), target_n_queries=target)
        res["global_steps"] = np.array(r.steps_per_iter, np.int64)
        res["global_onestep"] = np.array([r.onestep_from_iter, r.onestep_iterations], np.int64)
        res["band"] = r.download("final_rgba")[r0:r1]
        eng.detach_comm()
        if rank == 0:   # the single-GPU frame
            fresh()
            r = eng.frame(target_n_queries=target)
            res["full_steps"] = np.array(r.steps_per_iter, np.int64)
            res["full_onestep"] = np.array([r.onestep_from_iter, r.onestep_iterations], np.int64)
            res["full"] = r.download("final_rgba")
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
        tb.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bounds,overrides,config,target", [
    ([0, 540, 1080], {}, "c3", TARGET),
    ([0, 301, 777, 1080], {}, "c3", TARGET),
    ([0, 301, 1080], {"res_factor": 16}, "c3", TARGET),   # NeRF at half resolution: bands split NeRF rows by ceil(y / 2)
    # C4 at the reference's 2^21 target: ~1100 one-step iterations, marched by the ray-local one-step regime
    # (fused.hip) whose length comes from the death histograms summed over the ranks
    ([0, 500, 1080], {"show_virtual_obj": 0, "shadow_on_nerf": 0}, "c4", 0),
], ids=["even2", "uneven3", "halfres2", "c4_onestep2"])
def test_bands_with_global_schedule_equal_single_gpu(bounds, overrides, config, target):
    import torch.multiprocessing as mp
    world = len(bounds) - 1
    ctx = mp.get_context("spawn")
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        procs = [ctx.Process(target=_band_worker, args=(r, world, port, bounds, overrides, d, config, target)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=400)
        codes = [p.exitcode for p in procs]
        for p in procs:
            if p.exitcode is None:
                p.kill()
        assert codes == [0] * world, codes
        res = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(world)]
    full = res[0]["full"]
    for r in range(world):
        r0, r1 = bounds[r], bounds[r + 1]
        # the frame-wide schedule is the single-GPU one ...
        assert _prefix_equal(res[r]["global_steps"], res[0]["full_steps"])
        # ... and the band equals the single-GPU frame's rows bit for bit
        assert np.array_equal(res[r]["band"].view(np.uint32), full[r0:r1].view(np.uint32)), f"rank {r}"
        if config == "c4":   # the regime ran, with the single-GPU frame's length
            assert res[r]["global_onestep"][1] > 100 and np.array_equal(res[r]["global_onestep"], res[0]["full_onestep"])
    # without the exchange the bands step differently (the check above is not vacuous)
    assert any(not _prefix_equal(res[r]["local_steps"], res[0]["full_steps"]) for r in range(world))


@pytest.mark.parametrize("config,target", [("c3", TARGET), ("c4", 0)])
def test_rccl_schedule_world1_matches_local(config, target):
    """sng_set_comm at world size 1: RCCL all-reduce of the count on the NeRF stream (C4: and of the one-step
    regime's death histogram)."""
    import ctypes
    from synerfgine_amd import _lib
    from synerfgine_amd import scene as S
    tb, eng, _ = S.make_engine(config)
    try:
        rng = [eng.rng_states(0), eng.rng_states(1)]

        def fresh():
            eng.set_rng_states(0, rng[0])
            eng.set_rng_states(1, rng[1])

        fresh()
        a = eng.frame(target_n_queries=target)
        if config == "c4":
            assert a.onestep_iterations > 100
        ref = a.download("final_rgba")
        lib = eng._lib
        uid = (ctypes.c_uint8 * _lib.SNG_COMM_ID_BYTES)()
        _lib.check(lib.sng_comm_unique_id(uid))
        _lib.check(lib.sng_set_comm(eng.ctx, uid, 0, 1))
        fresh()
        b = eng.frame(target_n_queries=target)
        got = b.download("final_rgba")
        assert list(b.steps_per_iter) == list(a.steps_per_iter)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        # a host reducer cannot be attached on top of a communicator
        with pytest.raises(_lib.SngError):
            eng.attach_host_reducer(lambda v: v)
        eng.detach_comm()
        fresh()
        c = eng.frame(target_n_queries=target)
        assert np.array_equal(c.download("final_rgba").view(np.uint32), ref.view(np.uint32))
    finally:
        tb.close()


def _fresh_fn(eng):
    rng = [eng.rng_states(0), eng.rng_states(1)]

    def fresh():
        eng.set_rng_states(0, rng[0])
        eng.set_rng_states(1, rng[1])
    return fresh


@pytest.mark.parametrize("config,target,bands", [
    ("c3", TARGET, [(0, 301), (301, 777), (777, 1080)]),
    ("c4", 0, [(0, 500), (500, 1080), (420, 560)]),
], ids=["c3_small_target", "c4_onestep_msr"])
def test_schedule_replay_band_equals_single_gpu_rows(config, target, bands):
    """sng_set_sched_replay: the full frame's reduced values (recorded by a world-size-1 host reducer) replayed at
    every reduction point of a band reproduce that band as a rank under sng_set_comm renders it -- the single-GPU
    frame's rows bit for bit -- with the same number of reductions and no communicator (tools/band8.py times bands
    this way).  Two frames: the first from cleared step hints, the second from the hints the first one wrote."""
    from synerfgine_amd import _lib
    from synerfgine_amd import scene as S
    overrides = {"show_virtual_obj": 0, "shadow_on_nerf": 0} if config == "c4" else {}
    tb, eng, _ = S.make_engine(config, overrides=overrides)
    try:
        fresh = _fresh_fn(eng)
        fresh()
        local = eng.frame(target_n_queries=target).download("final_rgba")
        log = eng.record_schedule()
        recs, fulls = [], []
        for _ in range(2):
            fresh()
            r = eng.frame(target_n_queries=target)
            recs.append(list(log))
            log.clear()
            fulls.append(r.download("final_rgba"))
            assert r.sched_reductions == len(recs[-1]) > 0
        eng.detach_comm()
        if config == "c4":
            assert r.onestep_iterations > 100 and r.msr_rounds >= 1, (r.onestep_iterations, r.msr_rounds)
        # the frame-wide schedule at world size 1 is the local one
        assert np.array_equal(fulls[0].view(np.uint32), local.view(np.uint32))
        assert np.array_equal(fulls[1].view(np.uint32), local.view(np.uint32))
        for (r0, r1) in bands:
            for k in range(2):
                eng.set_sched_replay(recs[k])
                fresh()
                b = eng.frame(rows=(r0, r1), target_n_queries=target)
                assert b.sched_reductions == len(recs[k])
                got = b.download("final_rgba")[r0:r1]
                assert np.array_equal(got.view(np.uint32), fulls[k][r0:r1].view(np.uint32)), (r0, r1, k)
            eng.set_sched_replay(None)
        # records that do not match the frame's reductions fail loudly
        eng.set_sched_replay(recs[1][:-1])
        fresh()
        with pytest.raises(_lib.SngError):
            eng.frame(rows=bands[0], target_n_queries=target)
        eng.set_sched_replay(None)
    finally:
        tb.close()


def _msr_band_worker(rank, world, port, bounds, out_dir, target):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from synerfgine_amd import scene as S
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tb, eng, _ = S.make_engine("c4", overrides={"show_virtual_obj": 0, "shadow_on_nerf": 0})

        def reduce_fn(vals):
            t = torch.tensor(vals, dtype=torch.int64)
            dist.all_reduce(t)
            return t.tolist()

        fresh = _fresh_fn(eng)
        r0, r1 = bounds[rank], bounds[rank + 1]
        res = {}
        # two band-local frames first: each rank's step hints are its own band's (they differ across ranks)
        for _ in range(2):
            fresh()
            r = eng.frame(rows=(r0, r1), target_n_queries=target)
        res["local_msr"] = np.array([r.msr_rounds], np.int64)
        eng.attach_host_reducer(reduce_fn)
        bands = []
        for _ in range(2):
            fresh()
            r = eng.frame(rows=(r0, r1), target_n_queries=target)
            bands.append(r.download("final_rgba")[r0:r1])
        res["global_msr"] = np.array([r.msr_rounds], np.int64)
        res["band0"], res["band1"] = bands
        eng.detach_comm()
        if rank == 0:
            fresh()
            res["full"] = eng.frame(target_n_queries=target).download("final_rgba")
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
        tb.close()
    finally:
        dist.destroy_process_group()


def test_msr_rounds_after_local_frames_stay_frame_wide():
    """the multi-step rounds size K from the last frame's step hints.  After band-local frames the
    ranks' hints differ; attaching the reducer clears them, so every rank forms the same K and the global bands
    still equal the single-GPU rows (a divergent K would hang the exchange or break the equality)."""
    import torch.multiprocessing as mp
    bounds = [0, 500, 1080]
    world = 2
    ctx = mp.get_context("spawn")
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        procs = [ctx.Process(target=_msr_band_worker, args=(r, world, port, bounds, d, 0)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=400)
        codes = [p.exitcode for p in procs]
        for p in procs:
            if p.exitcode is None:
                p.kill()
        assert codes == [0] * world, codes
        res = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(world)]
    full = res[0]["full"]
    for r in range(world):
        assert res[r]["local_msr"][0] >= 1 and res[r]["global_msr"][0] >= 1, (res[r]["local_msr"], res[r]["global_msr"])
        for k in ("band0", "band1"):
            assert np.array_equal(res[r][k].view(np.uint32), full[bounds[r]:bounds[r + 1]].view(np.uint32)), (r, k)


def test_rccl_gather_rgba8_world1_equals_final_rgba8():
    """sng_gather_rgba8 (comm.cpp comm_gather_to_root) at world size 1: the rank-0 local band copy lands at the band's
    row offset and the received frame equals sng_final_rgba8 of the full frame byte for byte; bounds that do not
    tile [0, height) are rejected.  (Reference copy-back: testbed.cu:5126-5127.)"""
    import ctypes
    import torch
    from synerfgine_amd import _lib
    from synerfgine_amd import scene as S
    tb, eng, _ = S.make_engine("c3", width=320, height=180)
    try:
        lib = eng._lib
        uid = (ctypes.c_uint8 * _lib.SNG_COMM_ID_BYTES)()
        _lib.check(lib.sng_comm_unique_id(uid))
        _lib.check(lib.sng_set_comm(eng.ctx, uid, 0, 1))
        eng.frame()
        W, H = eng.resolution()["mesh"]
        frame = torch.full((H, W), -1, dtype=torch.int32, device="cuda")
        ref = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        eng.gather_rgba8([0, H], frame.data_ptr())
        _lib.check(lib.sng_synchronize(eng.ctx))
        _lib.check(lib.sng_final_rgba8(eng.ctx, 0, H, ctypes.c_void_p(ref.data_ptr()), None))
        _lib.check(lib.sng_synchronize(eng.ctx))
        torch.cuda.synchronize()
        assert torch.equal(frame, ref)
        assert int((ref != 0).sum()) > 0
        # the RGBA8 words are the final frame's unorm8 encoding
        fin = eng.frame().download("final_rgba")
        _lib.check(lib.sng_final_rgba8(eng.ctx, 0, H, ctypes.c_void_p(ref.data_ptr()), None))
        _lib.check(lib.sng_synchronize(eng.ctx))
        got = ref.cpu().numpy().view(np.uint8).reshape(H, W, 4).astype(np.int32)
        want = np.clip(np.rint(np.clip(fin, 0.0, 1.0) * 255.0), 0, 255).astype(np.int32)
        assert np.abs(got - want).max() <= 1
        for bad in ([0, H - 1], [1, H], [0, H + 1]):
            with pytest.raises(_lib.SngError):
                eng.gather_rgba8(bad, frame.data_ptr())
        eng.detach_comm()
        with pytest.raises(_lib.SngError):   # no communicator attached
            eng.gather_rgba8([0, H], frame.data_ptr())
    finally:
        tb.close()


@pytest.mark.parametrize("rows", [(501, 560), (380, 396), (0, 60)], ids=["object_band", "thin16", "sky_band"])
def test_fused_shadow_band_equals_separate_shadow_kernel(rows):
    """rt_fused_shadow: a thin band whose tiles all fit the path kernel's first round has its shadow rays traced by the
    path kernel's idle waves (a workgroup-local LDS queue of record allocations, mesh.hip fq_publish / fq_consume)
    instead of shadow_rays_kernel.  The band's frame buffers and the mesh XORWOW states the frame leaves are the same
    bits either way."""
    from synerfgine_amd import scene as S
    tb, eng, _ = S.make_engine("c3")
    try:
        fresh = _fresh_fn(eng)
        out = {}
        for fused in (0, 1):
            eng.set_param("rt_fused_shadow", fused)
            for k in range(2):   # a second frame: tile order and wave priorities from the first one's costs
                fresh()
                r = eng.frame(rows=rows, target_n_queries=TARGET)
            assert eng.get_param("rt_fused_shadow_used") == fused
            out[fused] = {b: r.download(b)[rows[0]:rows[1]].copy() for b in ("final_rgba", "syn_rgba", "syn_depth")}
            out[fused]["rng"] = eng.rng_states(1).copy()
        for b in out[0]:
            assert np.array_equal(out[0][b].view(np.uint32), out[1][b].view(np.uint32)), b
    finally:
        tb.close()


@pytest.mark.parametrize("config", ["c3", "c4"])
def test_rt_first_is_scheduling_only(config):
    """rt_first: on concurrent frames the NeRF stream waits on the device (bounded) for the path kernel's first workgroup
    before init_rays.  It changes only when work lands on the CUs: the frame buffers and the RNG states are the same bits
    with and without it, over two frames."""
    from synerfgine_amd import scene as S
    tb, eng, _ = S.make_engine(config, width=480, height=270, model="lego" if config == "c3" else "synthetic")
    try:
        fresh = _fresh_fn(eng)
        out = {}
        for on in (0, 1):
            eng.set_param("rt_first", on)
            fresh()
            for k in range(2):
                r = eng.frame(target_n_queries=TARGET if config == "c3" else 0)
            out[on] = {b: r.download(b).copy() for b in ("final_rgba", "syn_rgba", "syn_depth", "nerf_rgba")}
            out[on]["rng0"] = eng.rng_states(0).copy()
            out[on]["rng1"] = eng.rng_states(1).copy()
        for b in out[0]:
            assert np.array_equal(out[0][b].view(np.uint32), out[1][b].view(np.uint32)), b
    finally:
        tb.close()
