"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel count/total/avg, plus the launch sequence of one kernel.

usage: python tools/kernel_table.py <kernel_trace.csv> [substring-for-sequence] [max-seq]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("sng::", "")


def main():
    path = sys.argv[1]
    seq_key = sys.argv[2] if len(sys.argv) > 2 else None
    max_seq = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(lambda: [0, 0.0])
    seq = []
    for r in rows:
        k = short(r["Kernel_Name"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        agg[k][0] += 1
        agg[k][1] += dur
        if seq_key and seq_key in k:
            seq.append(dur)
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':60s} {'calls':>7s} {'total_us':>12s} {'avg_us':>10s} {'pct':>6s}")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k[:60]:60s} {n:7d} {t:12.1f} {t / n:10.2f} {100 * t / tot:6.2f}")
    if seq:
        print(f"sequence of '{seq_key}' ({len(seq)} launches, us):")
        print(" ".join(f"{d:.0f}" for d in seq[:max_seq]))


if __name__ == "__main__":
    main()
