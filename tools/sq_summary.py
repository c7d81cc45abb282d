"""VALU roofline of the hot kernels from one rocprofv3 pass: --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE with --kernel-trace (durations).

VALU peak (MI355X_MICROARCH.md, "Wave scheduling"): a SIMD issues one wave64 VALU instruction per 2 cycles
(32 lanes/cycle), 4 SIMDs per CU, 256 CUs, 2.4 GHz -> 1.229e12 wave-instructions/s.  A packed-f32 instruction
(v_pk_*) counts once.  valu_frac = SQ_INSTS_VALU per launch / (launch duration x peak rate); the durations come
from the same (serialising) counter pass, so they are those of kernels running alone.
usage: python tools/sq_summary.py <pass dir> <out.json> [config]
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

PEAK_WAVE_INSTR_PER_S = 256 * 4 * 0.5 * 2.4e9
KEYS = ("raytrace_kernel", "raytrace_pl_kernel", "shadow_rays_kernel", "rt_record_colour_kernel", "rt_accumulate_kernel", "rt_shade_records_kernel",
        "nerf_network_kernel", "spec_generate_kernel", "spec_composite_kernel", "init_rays_kernel", "generate_kernel", "nerf_fused_kernel",
        "shade_shadow_kernel", "shadow_draw_kernel", "shadow_term_kernel", "shadow_finish_kernel", "msr_generate_kernel", "msr_count_kernel",
        "msr_commit_kernel", "nerf_onestep_kernel", "onestep_schedule_kernel", "train_generate_kernel", "train_field_kernel",
        "train_loss_kernel", "train_dloss_kernel", "train_dw_kernel", "train_adam_kernel")


def short(n):
    return re.sub(r"\(.*", "", n).replace("void ", "").replace("sng::", "")


def main():
    d, out = sys.argv[1], sys.argv[2]
    cfg = sys.argv[3] if len(sys.argv) > 3 else "c3"
    cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not cc:
        raise SystemExit("no counter_collection.csv under " + d)
    per = defaultdict(lambda: defaultdict(float))     # (kernel) -> counter -> sum
    disp = defaultdict(set)
    for r in csv.DictReader(open(cc[0])):
        k = short(r["Kernel_Name"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    dur = defaultdict(list)
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    res = {}
    for key in KEYS:
        ks = [k for k in per if k.split("<")[0] == key or (k.startswith("_Z") and key in k)]
        if not ks:
            continue
        n = sum(len(disp[k]) for k in ks)
        tot = defaultdict(float)
        for k in ks:
            for c, v in per[k].items():
                tot[c] += v
        t = sum(sum(dur[k]) for k in ks)
        nd = sum(len(dur[k]) for k in ks)
        row = {"kernels": ks, "launches": n, **{c.lower() + "_per_launch": tot[c] / n for c in sorted(tot)}}
        if nd:
            avg = t / nd
            row["avg_launch_ms"] = avg * 1e3
            row["valu_frac"] = tot["SQ_INSTS_VALU"] / n / (avg * PEAK_WAVE_INSTR_PER_S)
            if tot.get("SQ_WAVE_CYCLES"):
                row["issue_cycles_per_wave_instr"] = tot["SQ_WAVE_CYCLES"] / max(1.0, tot["SQ_INSTS_VALU"] + tot["SQ_INSTS_SALU"] + tot["SQ_INSTS_LDS"])
        res[key] = row
    doc = {"note": "tools/sq_summary.py: SQ_INSTS_* per launch and the VALU roofline (peak 1.229e12 wave64 VALU instructions/s = 256 CUs x 4 SIMDs x 1/2 per cycle x 2.4 GHz); "
                   "durations from the counter pass's kernel trace (kernels serialised)", "config": cfg, "kernels": res}
    json.dump(doc, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:28s} launches {v['launches']:4d}  valu/launch {v.get('sq_insts_valu_per_launch', 0):12.4g}  ms {v.get('avg_launch_ms', 0):8.3f}  valu_frac {v.get('valu_frac', 0):.3f}")


if __name__ == "__main__":
    main()
