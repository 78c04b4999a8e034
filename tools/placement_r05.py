#!/usr/bin/env python3
"""Does plain streaming see the placement bands? (round 5)

One C2 bench stage (256-frame launches) whose placement search runs every
try (placement_flags=1): each candidate -- fresh arenas of 2 MiB pieces, or
with --plain fresh per-level hipMalloc rings -- is timed with the stage's
kernel and with the copy-third streaming probe into the same memory
(aqz_placement_report.probe_gbs).  One JSON line per stage.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "acquire-zarr_amd"))
import aqz  # noqa: E402

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tries", type=int, default=6)
    ap.add_argument("--plain", action="store_true")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--instances", type=int, default=1,
                    help="successive stages in this process, each closed before the next")
    a = ap.parse_args()
    c = bench.CONFIGS[a.config]
    B = a.batch or c["batch"]
    kw = dict(force_levels=c["force_levels"], max_batch_frames=B,
              layer_slots=bench.layer_slots_for(c, B), placement_tries=a.tries,
              placement_flags=1)
    if a.plain:
        kw["ring_malloc_flags"] = 0x10000
    for inst in range(a.instances):
        report(a, c, B, inst, kw)


def report(a, c, B, inst, kw):
    st = aqz.Stage(c["dims"], c["dtype"], c["method"], **kw)
    pl = st.placement()
    st.close()
    alg = pl["alg_bytes"]
    print(json.dumps({"config": a.config, "inst": inst, "plain": a.plain, "batch": B,
                      "mode": pl["mode"],
                      "stage_ms": pl["candidates_ms"],
                      "stage_bus_gbs": [round(alg / (m * 1e-3) / 1e9, 1)
                                        for m in pl["candidates_ms"]],
                      "probe_gbs": pl["candidates_probe_gbs"], "kept": pl["kept"],
                      "kept_ms_final": pl["kept_ms_final"],
                      "peak_gb": round(pl["peak_device_bytes"] / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
