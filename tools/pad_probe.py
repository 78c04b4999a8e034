#!/usr/bin/env python3
# HISTORICAL (rounds 2-3): the AQZ_* environment switches this probe sets were
# removed in round 4 (kernel tuning is only in aqz_stage_bench_options, e.g.
# aqz.Stage(..., knobs=..., chunk_pad_bytes=...)); kept for the provenance of
# the profiles/ files it produced.
"""Dev probe (not product): does staggering the chunk pitch (AQZ_CHUNK_PAD)
remove the placement bands of the C2 stage kernel?  For every pad, S stages
are created and held together (S placements, creation-time search off),
each timed over `reps` 128-frame launches from a random 2 GiB source, two
rounds; then they are freed before the next pad.  Prints ms per launch per
stage and the spread per pad."""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))
os.environ["AQZ_PLACEMENT_TRIES"] = "1"

import aqz  # noqa: E402
import torch  # noqa: E402

SPACE, TIME = 0, 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pads", default="0,4096,16384,69632,270336,1052672,3149824")
    ap.add_argument("--stages", type=int, default=6)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--pyramid-only", action="store_true")
    ap.add_argument("--interleave", action="store_true",
                    help="create all stages up front, pads cycling, all held")
    args = ap.parse_args()
    B, H, W = args.batch, 2048, 2048
    fbytes = H * W * 2
    dev = torch.device("cuda", 0)
    src = torch.empty(2 * B * fbytes, dtype=torch.uint8, device=dev)
    src.view(torch.int16).random_(-32768, 32767)
    dims = [(TIME, 0, 64, 1), (SPACE, H, args.chunk, 1), (SPACE, W, args.chunk, 1)]
    if args.interleave:
        pads = args.pads.split(",")
        stages = []
        for i in range(args.stages * len(pads)):
            os.environ["AQZ_CHUNK_PAD"] = pads[i % len(pads)]
            stages.append((pads[i % len(pads)],
                           aqz.Stage(dims, 1, 1, max_batch_frames=B, layer_slots=2,
                                     force_levels=5, skip_level0_split=args.pyramid_only)))
        torch.cuda.synchronize()
        res = {p: [] for p in pads}
        for pad, st in stages:
            ts = []
            for rnd in range(2):
                st.append_ptr(src.data_ptr(), B)
                st.synchronize()
                st.timing_mark(0)
                for k in range(args.reps):
                    st.append_ptr(src.data_ptr() + (k % 2) * B * fbytes, B)
                st.timing_mark(1)
                ts.append(st.timing_elapsed() / args.reps)
            res[pad].append(min(ts))
        for pad in pads:
            best = res[pad]
            print(f"pad {int(pad):8d}: " + " ".join(f"{v:.4f}" for v in best) +
                  f"  | median {statistics.median(best):.4f} min {min(best):.4f} "
                  f"max {max(best):.4f}", flush=True)
        return
    for pad in args.pads.split(","):
        os.environ["AQZ_CHUNK_PAD"] = pad
        stages = [aqz.Stage(dims, 1, 1, max_batch_frames=B, layer_slots=2, force_levels=5,
                            skip_level0_split=args.pyramid_only)
                  for _ in range(args.stages)]
        torch.cuda.synchronize()
        best = []
        for st in stages:
            ts = []
            for rnd in range(2):
                st.append_ptr(src.data_ptr(), B)
                st.synchronize()
                st.timing_mark(0)
                for k in range(args.reps):
                    st.append_ptr(src.data_ptr() + (k % 2) * B * fbytes, B)
                st.timing_mark(1)
                ts.append(st.timing_elapsed() / args.reps)
            best.append(min(ts))
        print(f"pad {int(pad):8d}: " + " ".join(f"{v:.4f}" for v in best) +
              f"  | median {statistics.median(best):.4f} min {min(best):.4f} "
              f"max {max(best):.4f}", flush=True)
        for st in stages:
            st.close()
        del stages
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
