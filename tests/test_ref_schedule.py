"""The oracle's wavefront schedule against the reference's own executions.

tests/golden/ref_nvprof_schedule.json holds, per frame and wavefront iteration, the launch extents of the
reference CUDA renderer's NerfTracer::trace_alt (testbed_nerf.cu:2155-2277) as its 20 shipped nvprof traces
recorded them (docs/assets_sng/profiling/*.nvvp; extracted read-only by tools/ref_nvprof_schedule.py).  The
scene's snapshot is not in the container, so the per-pixel results cannot be compared -- but each launch extent
encodes the sizes the schedule chose, and those must follow the oracle's rule (orc_wavefront_schedule):

  n_alive in (128 (gen - 1), 128 gen]                        generate / composite grids (linear_kernel, 128 threads)
  n_steps = clamp(2^21 / n_alive, 1, 8)                       testbed_nerf.cu:2188-2190
  n_elements = next_multiple(n_alive n_steps, 256) = 128 sh  :2210 (kernel_sh, 128 threads)
  kernel_grid grid = (n_elements / 512, n_levels)            tcnn GridEncoding over the same batch
  5 GEMM launches per inference                              density MLP (2 layers) + rgb MLP (3 layers), nerf_network.h:113-130
  compact(k+1) = gen(k); the frame ends at a compaction that finds no ray alive, with i < MARCH_ITER throughout
"""
import ctypes
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
TARGET = 2 * 1024 * 1024
MARCH_ITER = 10000          # testbed_nerf.cu:47


@pytest.fixture(scope="module")
def traces():
    with open(os.path.join(HERE, "golden", "ref_nvprof_schedule.json")) as f:
        d = json.load(f)
    assert d["columns"] == ["compact", "gen", "grid_x", "grid_y", "sh", "gemms", "comp"]
    return d["traces"]


def schedule(oracle_lib, n_alive):
    n_alive = np.ascontiguousarray(n_alive, np.uint32)
    steps = np.zeros(n_alive.size, np.uint32)
    elems = np.zeros(n_alive.size, np.uint64)
    oracle_lib.lib().orc_wavefront_schedule(n_alive.ctypes.data_as(ctypes.c_void_p), n_alive.size, TARGET,
                                            steps.ctypes.data_as(ctypes.c_void_p), elems.ctypes.data_as(ctypes.c_void_p))
    return steps, elems


def test_traces_cover_every_frame(traces):
    assert len(traces) == 20
    n_frames = sum(len(fr) for fr in traces.values())
    n_iters = sum(len(f["iterations"]) for fr in traces.values() for f in fr)
    assert n_frames == 16 * 25 + 50 + 40 + 4 + 6
    assert n_iters > 10000


def test_every_iteration_follows_the_oracle_schedule(traces, oracle_lib):
    checked = 0
    for name, frames in traces.items():
        for fi, f in enumerate(frames):
            its = np.array(f["iterations"], np.int64).reshape(-1, 7)
            n_px = f["advance"] * 128                     # advance_pos_nerf over every camera ray (1280 x 720 here)
            assert f["init_grid"][0] * f["init_grid"][1] * 128 >= n_px
            compact, gen, grid_x, grid_y, sh, gemms, comp = its.T
            # every alive count the generate grid admits, against the recorded padded batch
            cand = (gen[:, None] - 1) * 128 + np.arange(1, 129)[None, :]
            valid = (cand >= 1) & (cand <= n_px)
            steps, elems = schedule(oracle_lib, np.where(valid, cand, 1).ravel())
            steps, elems = steps.reshape(cand.shape), elems.reshape(cand.shape)
            match = valid & (elems == (sh * 128)[:, None])
            assert match.any(axis=1).all(), (name, fi, np.nonzero(~match.any(axis=1))[0][:5])
            # the admitted alive counts agree on the step count (so the iteration's i advances by it)
            s_lo = np.where(match, steps, 99).min(axis=1)
            s_hi = np.where(match, steps, 0).max(axis=1)
            assert (s_lo == s_hi).all(), (name, fi)
            assert (grid_x == (sh * 128 + 511) // 512).all() and (grid_y == 16).all()      # L = 16 levels, F = 2 in these traces
            assert (gemms == 5).all()
            assert (comp == gen).all()
            assert (compact[1:] == gen[:-1]).all() and compact[0] * 128 >= n_px - 127
            assert (np.diff(gen) <= 0).all()                                          # rays only die
            # the loop: i = 1 + sum of the previous iterations' steps stays below MARCH_ITER, and the frame ends
            # with a compaction that found no ray alive (its grid = the last iteration's alive count)
            i_before = 1 + np.concatenate([[0], np.cumsum(s_lo)[:-1]])
            assert (i_before < MARCH_ITER).all()
            assert f["closing_compact"] == gen[-1]
            checked += len(its)
    assert checked > 10000


def test_schedule_rule_edges(oracle_lib):
    n = np.array([1, 2, 262144, 262145, 699050, 699051, 1048576, 1048577, 2097152, 2097153, 2073600], np.uint32)
    steps, elems = schedule(oracle_lib, n)
    assert steps.tolist() == [8, 8, 8, 7, 3, 2, 2, 1, 1, 1, 1]
    assert (elems % 256 == 0).all() and (elems >= n.astype(np.uint64) * steps).all() and (elems - n.astype(np.uint64) * steps < 256).all()


def test_the_check_discriminates(traces):
    """The traces pin the rule: neighbouring rules (another query target, 128-padding) are
    contradicted by the recorded batches, and the recorded step counts span 2..8 (these 1280 x 720 frames start
    below 2^20 alive rays, so the one-step end of the clamp is not exercised by the traces)."""
    def admits(target, gran, smin):
        bad = 0
        for frames in traces.values():
            for f in frames:
                its = np.array(f["iterations"], np.int64).reshape(-1, 7)
                gen, sh = its[:, 1], its[:, 4]
                cand = (gen[:, None] - 1) * 128 + np.arange(1, 129)[None, :]
                steps = np.clip(target // cand, smin, 8)
                elems = (cand * steps + gran - 1) // gran * gran
                bad += int((~(elems == (sh * 128)[:, None]).any(axis=1)).sum())
        return bad
    assert admits(TARGET, 256, 1) == 0
    assert admits(TARGET // 2, 256, 1) > 0
    assert admits(TARGET * 2, 256, 1) > 0
    assert admits(TARGET, 128, 1) > 0
    seen = set()
    for frames in traces.values():
        for f in frames:
            its = np.array(f["iterations"], np.int64).reshape(-1, 7)
            seen |= set(np.unique(np.clip(TARGET // (its[:, 1] * 128), 1, 8)).tolist())
    assert seen == {2, 3, 4, 5, 6, 7, 8}, seen
