"""Per-launch HBM bytes of the hot kernels from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB.  MI355X_MICROARCH.md (HBM [CDNA4]):
on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide coalesced reads -> x2; WRITE_SIZE is exact for
16-B-per-lane stores.  half_to_float_kernel (reads 2 B, writes 4 B per density-grid cell, 128^3
cells, runs once per model load) is reported beside as a calibration point.
usage: python tools/pmc_summary.py <pmc dir> <out.json> [config] [bench log of the FETCH pass]

With the bench log, the file also records the counted run's own network samples per launch and launches per
frame (its bench.py line), which bench.py compares with the timed line before it quotes the traffic.
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def short(n):
    return re.sub(r"\(.*", "", n).replace("void ", "").replace("sng::", "")


N_SIMD = 256 * 4
N_XCD = 8


def load(d, counter, sub=None):
    f = glob.glob(f"{d}/{sub or counter}/**/*counter_collection.csv", recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv for {counter}")
    per = defaultdict(list)
    for r in sorted(csv.DictReader(open(f[0])), key=lambda r: int(r.get("Dispatch_Id", 0) or 0)):
        if r.get("Counter_Name", counter) != counter:
            continue
        per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def main():
    d, out = sys.argv[1], sys.argv[2]
    fetch, write = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        fa = sum(f) / len(f) if f else 0.0
        wa = sum(w) / len(w) if w else 0.0
        kernels[k] = {"launches": len(f), "fetch_kib_raw_avg": fa, "write_kib_avg": wa,
                      "hbm_bytes_per_launch": 2.0 * fa * 1024 + wa * 1024}
    # per-launch HBM bytes of the kernels bench.py reports, keyed by plain name (launch-weighted over variants)
    roof = {}
    for key in ("nerf_network_kernel", "nerf_fused_kernel", "nerf_onestep_kernel", "generate_kernel", "composite_kernel", "raytrace_kernel",
                "shadow_rays_kernel", "rt_accumulate_kernel", "shade_shadow_kernel", "init_rays_kernel", "shadow_term_kernel",
                "msr_generate_kernel", "msr_commit_kernel", "train_field_kernel", "train_dw_kernel", "train_generate_kernel",
                "train_adam_kernel", "train_loss_kernel"):
        ks = [k for k in kernels if key in k]
        n = sum(kernels[k]["launches"] for k in ks)
        if not n:
            continue
        fetch = sum(2.0 * kernels[k]["fetch_kib_raw_avg"] * 1024 * kernels[k]["launches"] for k in ks) / n
        wr = sum(kernels[k]["write_kib_avg"] * 1024 * kernels[k]["launches"] for k in ks) / n
        roof[key] = {"launches": n, "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": wr, "hbm_bytes_per_launch": fetch + wr}
    # launch durations from the FETCH pass's kernel trace (kernels serialised by the counter pass) -> byte rates.
    # FETCH_SIZE counts what the L2 (TCC) fetched from below it: the 256 MB Infinity Cache (MALL) serves part of
    # it, so a rate above the 8 TB/s HBM peak means MALL hits, not HBM traffic.
    dur = defaultdict(list)
    for f in glob.glob(f"{d}/FETCH_SIZE/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    for key, v in roof.items():
        ks = [k for k in dur if key in k]
        n = sum(len(dur[k]) for k in ks)
        if n:
            t = sum(sum(dur[k]) for k in ks) / n
            v["avg_launch_ms"] = t * 1e3
            v["below_l2_bytes_per_s"] = v["hbm_bytes_per_launch"] / t
            v["label"] = ("exceeds the HBM peak: part of FETCH_SIZE was served by the Infinity Cache (MALL)" if v["hbm_bytes_per_launch"] / t > 8e12
                          else "L2 fetch + write bytes (HBM or MALL)")
    net = [k for k in kernels if "nerf_network_kernel" in k]
    res = {"note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KiB->bytes; averages over all launches of bench.py --steps 3 --warmup 2 (the network kernel's roofline entry and hbm_bytes_per_launch: the timed frames' launches only); "
                   "FETCH_SIZE = bytes the L2 fetched from the Infinity Cache or HBM, so these are upper bounds on HBM traffic",
           "kernel": net[0] if net else None,
           "hbm_bytes_per_launch": kernels[net[0]]["hbm_bytes_per_launch"] if net else None,
           "calibration_half_to_float": dict(kernels.get("half_to_float_kernel", {}), expected_read_bytes=2 * 128 ** 3,
                                             expected_write_bytes=4 * 128 ** 3),
           "kernels": kernels, "roofline_kernels": roof, "config": sys.argv[3] if len(sys.argv) > 3 else None}
    # optional third pass: MFMA counters (SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F16, GRBM_GUI_ACTIVE)
    if glob.glob(f"{d}/MFMA/**/*counter_collection.csv", recursive=True) and net:
        busy, mops, gui = (load(d, c, "MFMA").get(net[0], []) for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_F16", "GRBM_GUI_ACTIVE"))
        avg = lambda v: sum(v) / len(v) if v else None
        b, m, g = avg(busy), avg(mops), avg(gui)
        res["mfma"] = {"launches": len(busy), "busy_cycles_avg": b, "mops_f16_avg": m, "flop_per_launch": m * 512 if m else None,
                       "gui_active_cycles_avg": g, "n_simd": N_SIMD, "n_xcd": N_XCD,
                       "kernel_cycles": g / N_XCD if g else None,
                       "mfma_busy_frac": b / (g / N_XCD * N_SIMD) if b and g else None,
                       "note": "GRBM_GUI_ACTIVE is the sum over the 8 XCDs (137 K cycles = the 57 us launch at 2.4 GHz); "
                               "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES (16 per v_mfma_f32_16x16x32_f16, summed over SIMDs) / "
                               "(kernel cycles x 1024 SIMDs); flop = MOPS_F16 x 512 (= samples x 20,480, SURVEY 8d)"}
    # MFMA pass, every kernel: busy fraction and flop per launch (the training GEMMs as well as the network)
    if glob.glob(f"{d}/MFMA/**/*counter_collection.csv", recursive=True):
        busy, mops, gui = (load(d, c, "MFMA") for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_F16", "GRBM_GUI_ACTIVE"))
        per = {}
        for k in busy:
            b, m, g = busy[k], mops.get(k, []), gui.get(k, [])
            if not b or not g or not sum(m):
                continue
            ba, ma, ga = sum(b) / len(b), sum(m) / len(m), sum(g) / len(g)
            per[k] = {"launches": len(b), "flop_per_launch": ma * 512, "mfma_busy_frac": ba / (ga / N_XCD * N_SIMD) if ga else None,
                      "mfma_tflops": ma * 512 / (ga / N_XCD / 2.4e9) / 1e12 if ga else None}
        res["mfma_per_kernel"] = per
    if len(sys.argv) > 4:   # the counted run's own bench line: samples per network launch, launches per frame
        line = None
        for l in open(sys.argv[4]):
            if l.startswith('{"metric"'):
                line = json.loads(l)
        if line:
            rf = line["roofline"]
            res["bench_line"] = {"samples_per_launch": rf["samples_in_launches"] / max(1, rf["launches"]),
                                 "launches_per_frame": rf["launches"] / max(1, line["steps"]), "steps": line["steps"],
                                 "warmup": line["warmup"], "workload": line["config"]["workload"]}
            if "nerf_network_kernel" in roof and net:
                v = roof["nerf_network_kernel"]
                # the timed frames' launches only (the last steps x launches-per-frame in dispatch order): the warm-up
                # frames march without the look-ahead hints, so their launches are larger than the line's
                n_t = int(round(rf["launches"]))
                f_all, w_all = load(d, "FETCH_SIZE").get(net[0], []), load(d, "WRITE_SIZE").get(net[0], [])
                if 0 < n_t <= min(len(f_all), len(w_all)):
                    f_t, w_t = f_all[-n_t:], w_all[-n_t:]
                    v["fetch_bytes_per_launch"] = 2.0 * sum(f_t) / n_t * 1024
                    v["write_bytes_per_launch"] = sum(w_t) / n_t * 1024
                    v["hbm_bytes_per_launch"] = v["fetch_bytes_per_launch"] + v["write_bytes_per_launch"]
                    v["launches_timed"] = n_t
                    res["hbm_bytes_per_launch"] = v["hbm_bytes_per_launch"]
                v["samples_per_launch"] = res["bench_line"]["samples_per_launch"]
                v["algorithmic_bytes_per_launch"] = v["samples_per_launch"] * (28 + 8 * 8 * 4 * 2 + 8)
                v["traffic_over_algorithmic"] = v["hbm_bytes_per_launch"] / v["algorithmic_bytes_per_launch"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * max(1, kv[1]["launches"]))[:12]:
        print(f"{k[:60]:60s} n={v['launches']:4d} fetch={v['fetch_kib_raw_avg']:12.1f}KiB write={v['write_kib_avg']:12.1f}KiB")


if __name__ == "__main__":
    main()
