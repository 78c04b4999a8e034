#!/usr/bin/env python3
"""Dev probe (not product): does the placement band follow the rings'
offsets inside ONE allocation?  Every level's ring is carved from one
arena (bench option ring_arena_bytes; ring_malloc_flags 4 = physically
contiguous), and aqz_stage_bench_set_ring_offset moves all of them together
inside the same memory.  Same stage, same source, same arena: if the launch
time changes with the offset, the band is a function of where the rings sit
relative to each other / to the source, not of which allocation they are.
Prints ms per launch per offset (best of `rounds`) per stage."""
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
    ap.add_argument("--config", default="c2")
    ap.add_argument("--stages", type=int, default=2)
    ap.add_argument("--slack-mib", type=int, default=512)
    ap.add_argument("--flags", type=int, default=4)
    ap.add_argument("--offsets-kib", default="0,4,64,256,1024,2048,3072,4096,8192,"
                                            "16384,65536,131072,262144,524288")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    c = bench.CONFIGS[args.config]
    B = c["batch"]
    h, w = c["dims"][-2][1], c["dims"][-1][1]
    fbytes = h * w * bench.BPP[c["dtype"]]
    nb = max(1, c["ring"] // B)
    src = torch.empty(nb * B * fbytes, dtype=torch.uint8, device="cuda")
    bench.fill_ring(torch, src, c["dtype"], 77)
    torch.cuda.synchronize()
    offs = [int(x) * 1024 for x in args.offsets_kib.split(",")]
    offs = [o for o in offs if o <= args.slack_mib << 20]
    for s in range(args.stages):
        st = aqz.Stage(c["dims"], c["dtype"], c["method"], max_batch_frames=B,
                       layer_slots=bench.layer_slots_for(c, B),
                       force_levels=c["force_levels"], ring_arena_bytes=args.slack_mib << 20,
                       ring_malloc_flags=args.flags)
        best = {}
        for _ in range(args.rounds):
            for o in offs:
                st.set_ring_offset(o)
                for i in range(2):
                    st.append_ptr(src.data_ptr() + (i % nb) * B * fbytes, B)
                st.synchronize()
                st.timing_mark(0)
                for i in range(args.reps):
                    st.append_ptr(src.data_ptr() + (i % nb) * B * fbytes, B)
                st.timing_mark(1)
                ms = st.timing_elapsed() / args.reps
                best[o] = min(best.get(o, 1e9), ms)
        print(f"{args.config} stage{s} " +
              " ".join(f"{o // 1024}K={best[o]:.4f}" for o in offs), flush=True)
        st.close()


if __name__ == "__main__":
    main()
