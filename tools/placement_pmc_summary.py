#!/usr/bin/env python3
"""Summarise tools/placement_pmc.py runs under rocprofv3 (dev tool).

usage: placement_pmc_summary.py OUTDIR [OUTDIR ...]
Each OUTDIR holds probe.json (the probe's --out) and rocprofv3's
run_kernel_trace.csv / run_counter_collection.csv.  Prints, per stage, the
median kernel duration (kernel trace of the same process) and the median of
every collected counter over that stage's fused dispatches, sorted by
duration, plus each counter's rank correlation with duration.
"""
import csv
import glob
import json
import os
import statistics
import sys


def find(d, suffix):
    hits = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    return hits[0] if hits else None


def spearman(x, y):
    def ranks(v):
        o = sorted(range(len(v)), key=lambda i: v[i])
        r = [0] * len(v)
        for k, i in enumerate(o):
            r[i] = k
        return r
    rx, ry = ranks(x), ranks(y)
    n = len(x)
    if n < 3:
        return float("nan")
    d2 = sum((a - b) ** 2 for a, b in zip(rx, ry))
    return 1 - 6 * d2 / (n * (n * n - 1))


def one(d):
    probe = json.load(open(os.path.join(d, "probe.json")))
    order = probe["order"]
    kt = find(d, "kernel_trace.csv")
    cc = find(d, "counter_collection.csv")
    dur = {}
    if kt:
        for r in csv.DictReader(open(kt)):
            if "fused_pyramid" in r["Kernel_Name"]:
                dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) -
                                              int(r["Start_Timestamp"])) / 1e6
    ctr = {}
    if cc:
        for r in csv.DictReader(open(cc)):
            if "fused_pyramid" in r["Kernel_Name"]:
                ctr.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(
                    r["Counter_Value"])
    ids = sorted(set(dur) | set(ctr))
    if len(ids) != len(order):
        print(f"{d}: {len(ids)} fused dispatches, probe issued {len(order)}")
        ids = ids[-len(order):]
    per = {}
    for i, s in zip(ids, order):
        e = per.setdefault(s, {"ms": [], "c": {}})
        if i in dur:
            e["ms"].append(dur[i])
        for k, v in ctr.get(i, {}).items():
            e["c"].setdefault(k, []).append(v)
    rows = []
    for s, e in per.items():
        rows.append((s, statistics.median(e["ms"]) if e["ms"] else float("nan"),
                     {k: statistics.median(v) for k, v in e["c"].items()}))
    rows.sort(key=lambda r: r[1])
    names = sorted({k for r in rows for k in r[2]})
    print(f"== {d}")
    print("stage  ms      " + "  ".join(names))
    for s, ms, c in rows:
        print(f"{s:5d} {ms:.4f}  " + "  ".join(f"{c.get(k, float('nan')):.4g}" for k in names))
    for k in names:
        xs = [r[2].get(k, 0.0) for r in rows]
        print(f"  rank corr(ms, {k}) = {spearman([r[1] for r in rows], xs):+.2f}")


if __name__ == "__main__":
    for d in sys.argv[1:]:
        one(d)
