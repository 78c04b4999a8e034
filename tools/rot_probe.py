#!/usr/bin/env python3
# HISTORICAL (rounds 2-3): the AQZ_* environment switches this probe sets were
# removed in round 4 (kernel tuning is only in aqz_stage_bench_options, e.g.
# aqz.Stage(..., knobs=..., chunk_pad_bytes=...)); kept for the provenance of
# the profiles/ files it produced.
"""Dev probe (not product): the XCD walk rotation (FusedParams.xcd_rot,
tuning knob bits 16-31) against placement bands.  S stages held together
(S placements, creation-time search off); every stage is timed under every
rotation, interleaved over rounds, so each placement is its own A/B.
Prints ms per launch, stage x rotation (min over rounds)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))
os.environ["AQZ_PLACEMENT_TRIES"] = "1"

import aqz  # noqa: E402
import torch  # noqa: E402

SPACE, TIME = 0, 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rots", default="0,8,256,264,512,520,1032")
    ap.add_argument("--knobs", default="", help="comma list of raw knob values (overrides --rots)")
    ap.add_argument("--stages", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--config", default="c2")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.config == "c4":
        B, H, W = 128, 2048, 2048
        dims = [(TIME, 0, 1, 1), (SPACE, 256, 64, 1), (SPACE, H, 256, 1), (SPACE, W, 256, 1)]
        kw = {}
        dt = 1
    else:
        B, H, W = 128, 2048, 2048
        dims = [(TIME, 0, 64, 1), (SPACE, H, 256, 1), (SPACE, W, 256, 1)]
        kw = {"force_levels": 5}
        dt = 1
    fbytes = H * W * 2
    src = torch.empty(2 * B * fbytes, dtype=torch.uint8, device=dev)
    src.view(torch.int16).random_(-32768, 32767)
    rots = [int(r) for r in args.rots.split(",")]
    knobs = [int(k) for k in args.knobs.split(",")] if args.knobs else [r << 16 for r in rots]
    stages = [aqz.Stage(dims, dt, 1, max_batch_frames=B, layer_slots=2, **kw)
              for _ in range(args.stages)]
    torch.cuda.synchronize()
    res = [[1e9] * len(knobs) for _ in stages]
    for rnd in range(args.rounds):
        for j, st in enumerate(stages):
            for i, kn in enumerate(knobs):
                st.set_tuning(kn, 7)
                st.append_ptr(src.data_ptr(), B)
                st.synchronize()
                st.timing_mark(0)
                for k in range(args.reps):
                    st.append_ptr(src.data_ptr() + (k % 2) * B * fbytes, B)
                st.timing_mark(1)
                res[j][i] = min(res[j][i], st.timing_elapsed() / args.reps)
    print("ms per launch; rows = stages (placements), cols = knobs " + str(knobs))
    for j, row in enumerate(res):
        print(f"stage{j} " + " ".join(f"{v:.4f}" for v in row), flush=True)
    cols = list(zip(*res))
    print("mean   " + " ".join(f"{sum(c) / len(c):.4f}" for c in cols))
    print("max    " + " ".join(f"{max(c):.4f}" for c in cols))


if __name__ == "__main__":
    main()
