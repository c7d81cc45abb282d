"""Extract the reference's own wavefront schedule from its nvprof traces (fixture generator, run in the build
container only: /root/reference does not exist on the GPU box).

The reference ships 20 nvprof traces of its CUDA renderer (`docs/assets_sng/profiling/*.nvvp`, SQLite files
written by nvprof).  They are opened read-only with sqlite3; nothing in them is executed.  For every frame of
every trace the NeRF stream's launches of `NerfTracer::trace_alt` (testbed_nerf.cu:2155-2277) are read in
order, and for each wavefront iteration this records the launch extents that encode its sizes:

  compact   compact_kernel_nerf grid.x            = ceil(n_alive_prev / 128)  (linear_kernel, 128 threads)
  gen       generate_next_nerf_network_inputs     = ceil(n_alive / 128)
  grid_x    tcnn kernel_grid grid.x               = ceil(n_elements / 512), grid.y = n_levels
  sh        tcnn kernel_sh grid.x                 = n_elements / 128, n_elements = next_multiple(n_alive * n_steps, 256)
  gemms     CUTLASS GEMM launches of the inference (the density and rgb MLPs' layers)
  comp      composite_kernel_nerf_alt grid.x      = ceil(n_alive / 128)

plus the frame's closing compaction (the one that finds no ray alive) and init_rays' / advance_pos' grids.
Output: tests/golden/ref_nvprof_schedule.json, checked by tests/test_ref_schedule.py against the oracle's
schedule rule (orc_wavefront_schedule: n_steps = clamp(2^21 / n_alive, 1, 8), testbed_nerf.cu:2188-2190, and
the 256-padding of :2210).

usage: python tools/ref_nvprof_schedule.py [--ref /root/reference] [--out tests/golden/ref_nvprof_schedule.json]"""
import argparse
import glob
import json
import os
import sqlite3

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_kind(name):
    if "compact_kernel_nerf" in name:
        return "compact"
    if "generate_next_nerf_network_inputs" in name:
        return "gen"
    if "kernel_grid" in name:
        return "grid"
    if "kernel_sh" in name:
        return "sh"
    if "cutlass" in name and "Gemm" in name:
        return "gemm"
    if "extract_density" in name:
        return "extract"
    if "composite_kernel_nerf_alt" in name:
        return "comp"
    if "ngp" in name and "init_rays_with_payload_kernel_nerf" in name:
        return "init"
    if "advance_pos_nerf_kernel" in name:
        return "advance"
    return None


def read_trace(path):
    con = sqlite3.connect(f"file:{path}?mode=ro", uri=True)
    try:
        cur = con.cursor()
        strings = dict(cur.execute("select _id_, value from StringTable"))
        rows = cur.execute("select start, streamId, gridX, gridY, blockX, name from CUPTI_ACTIVITY_KIND_CONCURRENT_KERNEL "
                           "order by start").fetchall()
    finally:
        con.close()
    launches = [(kernel_kind(strings[r[5]]), r[1], r[2], r[3], r[4]) for r in rows]
    launches = [l for l in launches if l[0] is not None]
    nerf_streams = {l[1] for l in launches if l[0] == "gen"}
    assert len(nerf_streams) == 1, nerf_streams
    s = nerf_streams.pop()
    seq = [l for l in launches if l[1] == s]
    frames, cur_f, it = [], None, None
    for kind, _, gx, gy, bx in seq:
        if kind == "init":
            it = None   # the previous frame's closing compaction ran no iteration
            cur_f = {"init_grid": [gx, gy], "advance": None, "iterations": [], "closing_compact": None}
            frames.append(cur_f)
            continue
        if cur_f is None:
            continue
        if kind == "advance":
            cur_f["advance"] = gx
        elif kind == "compact":
            assert bx == 128 and it is None, "a compaction inside an iteration"
            it = {"compact": gx}
            cur_f["closing_compact"] = gx
        elif kind == "gen":
            assert it is not None and "gen" not in it and bx == 128
            it["gen"] = gx
            cur_f["closing_compact"] = None
        elif kind == "grid":
            it["grid_x"], it["grid_y"] = gx, gy
        elif kind == "sh":
            assert bx == 128
            it["sh"] = gx
        elif kind == "gemm":
            it["gemms"] = it.get("gemms", 0) + 1
        elif kind == "comp":
            assert bx == 128
            it["comp"] = gx
            cur_f["iterations"].append(it)
            it = None
    return frames


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden", "ref_nvprof_schedule.json"))
    args = ap.parse_args()
    out = {"source": "reference docs/assets_sng/profiling/*.nvvp (nvprof SQLite traces of the CUDA renderer), read-only",
           "generator": "tools/ref_nvprof_schedule.py",
           "columns": ["compact", "gen", "grid_x", "grid_y", "sh", "gemms", "comp"], "traces": {}}
    for path in sorted(glob.glob(os.path.join(args.ref, "docs", "assets_sng", "profiling", "*.nvvp"))):
        frames = read_trace(path)
        enc = []
        for f in frames:
            its = [[i.get(c, -1) for c in out["columns"]] for i in f["iterations"]]
            enc.append({"init_grid": f["init_grid"], "advance": f["advance"], "closing_compact": f["closing_compact"], "iterations": its})
        out["traces"][os.path.basename(path)] = enc
        print(os.path.basename(path), len(frames), "frames,", sum(len(f["iterations"]) for f in frames), "iterations")
    with open(args.out, "w") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print("wrote", args.out, os.path.getsize(args.out), "bytes")


if __name__ == "__main__":
    main()
