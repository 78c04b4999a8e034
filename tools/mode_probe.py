#!/usr/bin/env python3
# HISTORICAL (rounds 2-3): the AQZ_* environment switches this probe sets were
# removed in round 4 (kernel tuning is only in aqz_stage_bench_options, e.g.
# aqz.Stage(..., knobs=..., chunk_pad_bytes=...)); kept for the provenance of
# the profiles/ files it produced.
"""Dev probe (not product): is the fast/slow mode of the C2 stage kernel a
property of the stage's own allocations, of the source ring, or of the
pair?  Creates S stages (bench C2 geometry, 128-frame launches) and R source
rings, times every (source, stage) pair, prints ms per launch as a matrix.
Env AQZ_MALLOC_FLAGS selects hipExtMallocWithFlags flags for the stages."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))

import aqz  # noqa: E402
import torch  # noqa: E402

SPACE, TIME = 0, 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stages", type=int, default=6)
    ap.add_argument("--sources", type=int, default=3)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--pyramid-only", action="store_true")
    args = ap.parse_args()
    B, H, W = args.batch, 2048, 2048
    fbytes = H * W * 2
    dev = torch.device("cuda", 0)
    srcs = []
    for r in range(args.sources):
        t = torch.empty(2 * B * fbytes, dtype=torch.uint8, device=dev)
        t.view(torch.int16).random_(-32768, 32767)
        srcs.append(t)
    dims = [(TIME, 0, 64, 1), (SPACE, H, 256, 1), (SPACE, W, 256, 1)]
    stages = [aqz.Stage(dims, 1, 1, max_batch_frames=B, layer_slots=2, force_levels=5,
                        skip_level0_split=args.pyramid_only)
              for _ in range(args.stages)]
    torch.cuda.synchronize()
    res = [[0.0] * args.stages for _ in srcs]
    for rnd in range(2):
        for i, s in enumerate(srcs):
            for j, st in enumerate(stages):
                for k in range(2):
                    st.append_ptr(s.data_ptr() + (k % 2) * B * fbytes, B)
                st.synchronize()
                st.timing_mark(0)
                for k in range(args.reps):
                    st.append_ptr(s.data_ptr() + (k % 2) * B * fbytes, B)
                st.timing_mark(1)
                ms = st.timing_elapsed() / args.reps
                res[i][j] = ms if rnd == 0 else min(res[i][j], ms)
    print("ms per %d-frame launch; rows = source rings, cols = stages" % B)
    for i, row in enumerate(res):
        print(f"src{i} " + " ".join(f"{v:.4f}" for v in row))
    for j, st in enumerate(stages):
        print(f"stage{j} placement {st.placement()}")


if __name__ == "__main__":
    main()
