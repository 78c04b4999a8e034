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

C2 = [(2, 0, 64, 1), (0, 2048, 256, 1), (0, 2048, 256, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tries", type=int, default=6)
    ap.add_argument("--plain", action="store_true")
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    kw = dict(force_levels=5, max_batch_frames=a.batch, layer_slots=max(2, a.batch // 64),
              placement_tries=a.tries, placement_flags=1)
    if a.plain:
        kw["ring_malloc_flags"] = 0x10000
    st = aqz.Stage(C2, 1, 1, **kw)
    pl = st.placement()
    st.close()
    alg = pl["alg_bytes"]
    print(json.dumps({"plain": a.plain, "batch": a.batch, "mode": pl["mode"],
                      "stage_ms": pl["candidates_ms"],
                      "stage_bus_gbs": [round(alg / (m * 1e-3) / 1e9, 1)
                                        for m in pl["candidates_ms"]],
                      "probe_gbs": pl["candidates_probe_gbs"], "kept": pl["kept"],
                      "kept_ms_final": pl["kept_ms_final"],
                      "peak_gb": round(pl["peak_device_bytes"] / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
