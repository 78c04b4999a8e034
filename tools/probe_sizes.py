#!/usr/bin/env python3
"""HBM probe rate against its launch size (round 5).

The live probe (aqz_probe_hbm) ran 512 MiB of input per launch, about 0.2 ms:
its ramp-up and drain are a larger share of a launch than in the stage's
0.77 ms C2 launches.  This sweeps the bytes per launch for the copy-third
shape (1 read : 4/3 write, the stage's) and the read shape, nontemporal and
plain stores, hipMalloc and 2 MiB pieces.  One JSON line per point.
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "acquire-zarr_amd"))
import aqz  # noqa: E402

WR = {aqz.PROBE_READ: 0.0, aqz.PROBE_COPY: 1.0, aqz.PROBE_COPY_THIRD: 4.0 / 3.0,
      aqz.PROBE_READ_THIRD: 1.0 / 3.0}
NAME = {aqz.PROBE_READ: "read", aqz.PROBE_COPY: "copy", aqz.PROBE_COPY_THIRD: "copy_third",
        aqz.PROBE_READ_THIRD: "read_third"}


def main():
    sizes = [int(s) << 20 for s in (sys.argv[1] if len(sys.argv) > 1 else
                                    "512,2048").split(",")]
    flavs = [p | k | d for p in (0, aqz.PROBE_PLAIN_STORES) for k in (0, aqz.PROBE_PIECES)
             for d in (0, aqz.PROBE_DEEP)]
    for shape in (aqz.PROBE_COPY_THIRD, aqz.PROBE_READ):
        for flav in ((0, aqz.PROBE_DEEP) if shape == aqz.PROBE_READ else flavs):
            for nb in sizes:
                reps = max(5, int(20 * (512 << 20) / nb))
                ms = []
                for _ in range(3):
                    t, rd = aqz.probe_hbm(shape | flav, nb, reps, 0)
                    ms.append(t)
                best = min(ms)
                print(json.dumps({"shape": NAME[shape], "plain": bool(flav & aqz.PROBE_PLAIN_STORES),
                                  "pieces": bool(flav & aqz.PROBE_PIECES),
                                  "deep": bool(flav & aqz.PROBE_DEEP), "mib": nb >> 20,
                                  "ms": round(best, 5),
                                  "bus_gbs": round(rd * (1 + WR[shape]) / (best * 1e-3) / 1e9, 1),
                                  "spread": round(max(ms) / best, 4)}), flush=True)


if __name__ == "__main__":
    main()
