#!/usr/bin/env python3
"""Summarise one tools/profile.sh output directory into profiles/.

Writes profiles/<tag>_<cfg>_pmc.json (per-launch HBM bytes of the dominant
kernel from the FETCH_SIZE / WRITE_SIZE passes, corrected as
MI355X_MICROARCH.md prescribes: FETCH_SIZE is in KiB and reports half the
bytes of a 16-B-per-lane streaming read on gfx950, so x2; WRITE_SIZE is in
KiB and exact) and copies the kernel-trace --stats table next to it.
bench.py reads the JSON for roofline.traffic.

usage: tools/pmc_summary.py gpurun_out/prof_r01_c2 c2 r01
"""
import csv
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out.setdefault(r["Kernel_Name"], {}).setdefault(r["Counter_Name"], []).append(
            float(r["Counter_Value"]))
    return out


def main():
    d, cfg, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    fpl = int(sys.argv[4]) if len(sys.argv) > 4 else None # frames per launch
    stats = list(csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))))
    ours = [s for s in stats if "aqz::" in s["Name"]]
    dom = max(ours, key=lambda s: float(s["TotalDurationNs"]))
    fetch = per_kernel(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(d, "pmc_write", "run_counter_collection.csv"))
    name = dom["Name"]
    f_kib = statistics.median(fetch[name]["FETCH_SIZE"])
    w_kib = statistics.median(write[name]["WRITE_SIZE"])
    res = {
        "config": cfg,
        "kernel": name,
        "launches_traced": int(dom["Calls"]),
        "avg_duration_ns": float(dom["AverageNs"]),
        "fetch_size_kib_median": f_kib,
        "write_size_kib_median": w_kib,
        "hbm_read_bytes_per_launch": int(f_kib * 1024 * 2),
        "hbm_write_bytes_per_launch": int(w_kib * 1024),
        "traffic_bytes_per_launch": int(f_kib * 1024 * 2 + w_kib * 1024),
        "correction": "FETCH_SIZE x2 (gfx950 reports half of a 16-B/lane streaming read); "
                      "KiB -> bytes",
    }
    if fpl:
        res["frames_per_launch"] = fpl
    # the library build that was profiled (bench.py prefers a summary of
    # the build it runs)
    shaf = os.path.join(d, "lib.sha256")
    if os.path.exists(shaf):
        res["lib_sha256"] = open(shaf).read().strip()
    # its device code (the .hip_fatbin section): builds that differ only in
    # host code share it (bench.py falls back to a summary of the same
    # device code); recorded when the profiled library is the one in-tree
    sys.path.insert(0, REPO)
    from bench import device_code_sha256, REPO as _r  # noqa: F401
    lib = os.path.join(REPO, "acquire-zarr_amd", "libaqz_gpu.so")
    import hashlib
    if res.get("lib_sha256") and os.path.exists(lib) and \
            hashlib.sha256(open(lib, "rb").read()).hexdigest() == res["lib_sha256"]:
        res["device_code_sha256"] = device_code_sha256(lib)
    # the traced bench line: how its rings were allocated (bench.py matches
    # a summary to a run by it) and its own event-timed kernel average
    try:
        line = [l for l in open(os.path.join(d, "bench_trace.log")) if l.startswith("{")][-1]
        b = json.loads(line)
        r = b["roofline"]
        res["ring_allocation"] = r["placement"]["ring_allocation"]
        res["bench_kernel_avg_ms"] = r["kernel_avg_ms"]
        res["bench_frac"] = r["frac"]
        cmd = os.path.join(d, "bench_cmd.txt")
        res["bench_command"] = (open(cmd).read().strip() if os.path.exists(cmd) else
                                "python3 bench.py --config %s --steps %s --warmup 5 "
                                "--no-cpu-baseline --no-pyramid-only-line --no-hbm-probe"
                                % (cfg, os.environ.get("STEPS", "200")))
        res["placement"] = {k: r["placement"].get(k) for k in
                            ("candidates_ms", "kept", "accepted", "expected_ms",
                             "probe_bus_gbs", "candidates_probe_gbs")}
    except (OSError, IndexError, KeyError, ValueError):
        pass
    # the timed launches alone: the stats average also holds the stage's
    # creation-time placement calibration (up to 10 launches per candidate)
    tr = os.path.join(d, "trace", "run_kernel_trace.csv")
    if os.path.exists(tr):
        steps = int(os.environ.get("STEPS", "200"))
        rows = sorted((r for r in csv.DictReader(open(tr)) if r["Kernel_Name"] == name),
                      key=lambda r: int(r["Start_Timestamp"]))
        dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows][-steps:]
        if dur:
            res["steady_avg_duration_ns"] = statistics.mean(dur)
            res["steady_launches"] = len(dur)
    sq = os.path.join(d, "pmc_sq", "run_counter_collection.csv")
    if os.path.exists(sq):
        s = per_kernel(sq).get(name, {})
        res["sq"] = {k: statistics.median(v) for k, v in s.items()}
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    base = os.path.join(REPO, "profiles", f"{tag}_{cfg}")
    with open(base + "_pmc.json", "w") as fh:
        json.dump(res, fh, indent=1)
    shutil.copy(os.path.join(d, "trace", "run_kernel_stats.csv"), base + "_kernel_stats.csv")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
