#!/usr/bin/env python3
"""Dev probe (not product): kernel-variant A/B on the SAME stage (same
placement) via aqz_stage_set_tuning(knobs, nt).  Knobs of the 2x2x2 path:
256 = the LDS-cascade fused_pyramid_3d, 512 = strip3d without the next-plane
prefetch.  Prints ms per launch (best of 2 rounds) per stage instance."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))

import aqz  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--instances", type=int, default=3)
    ap.add_argument("--knobs", default="0,512,256")
    ap.add_argument("--nt", type=int, default=7)
    ap.add_argument("--nts", default="", help="nontemporal policies to cross with --knobs")
    ap.add_argument("--pyramid-only", action="store_true",
                    help="stages without the level-0 split (skip_level0_split)")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--placement-tries", type=int, default=0)
    ap.add_argument("--xy", action="store_true", help="XY-transposed storage order")
    ap.add_argument("--batch", type=int, default=0, help="frames per launch (default: bench's)")
    ap.add_argument("--appends", default="",
                    help="append sizes (frames, dividing the batch) to compare on the same "
                         "stage: ms per batch of frames for each (with the first knob)")
    args = ap.parse_args()
    c = bench.CONFIGS[args.config]
    B = args.batch or c["batch"]
    h, w = c["dims"][-2][1], c["dims"][-1][1]
    fbytes = h * w * {0: 1, 1: 2, 8: 4}[c["dtype"]]
    src = torch.empty(2 * B * fbytes, dtype=torch.uint8, device="cuda")
    src.view(torch.int16).random_(-32768, 32767)
    # (two batches of frames: >= 2 GiB at the bench's batch sizes, past the
    # 256 MiB MALL)
    knobs = [int(x) for x in args.knobs.split(",")]
    nts = [int(x) for x in args.nts.split(",")] if args.nts else [args.nt]
    variants = [(k, t) for k in knobs for t in nts]
    nd = len(c["dims"])
    xy = dict(storage_order=list(range(nd - 2)) + [nd - 1, nd - 2]) if args.xy else {}
    for inst in range(args.instances):
        st = aqz.Stage(c["dims"], c["dtype"], c["method"], max_batch_frames=B,
                       layer_slots=bench.layer_slots_for(c, B), force_levels=c["force_levels"],
                       placement_tries=args.placement_tries,
                       skip_level0_split=args.pyramid_only, **xy)
        row = []
        for rnd in range(2):
            for j, (k, nt) in enumerate(variants):
                st.set_tuning(k, nt)
                for i in range(2):
                    st.append_ptr(src.data_ptr() + (i % 2) * B * fbytes, B)
                st.synchronize()
                st.timing_mark(0)
                for i in range(args.reps):
                    st.append_ptr(src.data_ptr() + (i % 2) * B * fbytes, B)
                st.timing_mark(1)
                ms = st.timing_elapsed() / args.reps
                row = row + [ms] if rnd == 0 else row
                row[j] = min(row[j], ms)
        extra = ""
        if args.appends:
            st.set_tuning(knobs[0], args.nt)
            sizes = [int(x) for x in args.appends.split(",")]
            best = {}
            for rnd in range(2):
                for a in sizes:
                    per = B // a
                    for i in range(2 * per):
                        st.append_ptr(src.data_ptr() + (i // per % 2) * B * fbytes +
                                      (i % per) * a * fbytes, a)
                    st.synchronize()
                    st.timing_mark(0)
                    for i in range(args.reps * per):
                        st.append_ptr(src.data_ptr() + (i // per % 2) * B * fbytes +
                                      (i % per) * a * fbytes, a)
                    st.timing_mark(1)
                    ms = st.timing_elapsed() / args.reps
                    best[a] = min(best.get(a, ms), ms)
            extra = " " + " ".join(f"append{a}={v:.4f}" for a, v in best.items())
        print(f"{args.config} B{B} inst{inst} {st.placement()['candidates_ms']} " +
              " ".join(f"k{k}/nt{t}={v:.4f}" for (k, t), v in zip(variants, row)) + extra, flush=True)
        st.close()


if __name__ == "__main__":
    main()
