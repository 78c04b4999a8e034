#!/usr/bin/env python3
# HISTORICAL (rounds 2-3): the AQZ_* environment switches this probe sets were
# removed in round 4 (kernel tuning is only in aqz_stage_bench_options, e.g.
# aqz.Stage(..., knobs=..., chunk_pad_bytes=...)); kept for the provenance of
# the profiles/ files it produced.
"""Dev probe (not product): what separates a fast chunk-ring placement from a
slow one?  Creates S stages of the bench C2 geometry in ONE process with the
creation-time search off (AQZ_PLACEMENT_TRIES=1), so each lands its rings
wherever the allocator puts them, then launches every stage R times in a
fixed order (stage 0's launches, then stage 1's, ...).  Run under
`rocprofv3 --pmc <counters> --kernel-trace`: dispatch order attributes every
fused-kernel dispatch to its stage, so per-stage counter medians can be set
against per-stage kernel durations of the same process (tools/placement_pmc_summary.py).
Without the profiler it prints per-stage event-timed ms per launch.

  --rounds N     repeat the per-stage sweep N times (placement stability)
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))
os.environ.setdefault("AQZ_PLACEMENT_TRIES", "1")

import aqz  # noqa: E402
import torch  # noqa: E402

SPACE, TIME = 0, 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stages", type=int, default=8)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--pyramid-only", action="store_true")
    ap.add_argument("--out", default="")
    ap.add_argument("--ballast-gib", type=int, default=0,
                    help="allocate and hold this much device memory first")
    args = ap.parse_args()
    B, H, W = args.batch, 2048, 2048
    fbytes = H * W * 2
    dev = torch.device("cuda", 0)
    ballast = [torch.empty(1 << 30, dtype=torch.uint8, device=dev)
               for _ in range(args.ballast_gib)]
    src = torch.empty(2 * B * fbytes, dtype=torch.uint8, device=dev)
    src.view(torch.int16).random_(-32768, 32767)
    dims = [(TIME, 0, 64, 1), (SPACE, H, 256, 1), (SPACE, W, 256, 1)]
    stages = [aqz.Stage(dims, 1, 1, max_batch_frames=B, layer_slots=2, force_levels=5,
                        skip_level0_split=args.pyramid_only)
              for _ in range(args.stages)]
    torch.cuda.synchronize()
    times = [[] for _ in stages]
    order = []  # stage of every fused dispatch, in dispatch order
    for rnd in range(args.rounds):
        for j, st in enumerate(stages):
            st.append_ptr(src.data_ptr(), B)  # warm-up
            order.append(j)
            st.synchronize()
            st.timing_mark(0)
            for k in range(args.reps):
                st.append_ptr(src.data_ptr() + (k % 2) * B * fbytes, B)
                order.append(j)
            st.timing_mark(1)
            times[j].append(st.timing_elapsed() / args.reps)
            st.synchronize()
    res = {"batch": B, "reps": args.reps, "rounds": args.rounds,
           "event_ms": times, "order": order,
           "kernel": stages[0].dominant_kernel()}
    for j, t in enumerate(times):
        print(f"stage{j} " + " ".join(f"{v:.4f}" for v in t))
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(res, fh)
    for st in stages:
        st.close()


if __name__ == "__main__":
    main()
