#!/usr/bin/env python3
"""Dev harness (not product): A/B kernel switches on the SAME stage, so the
allocation-dependent speed of a chunk-layer ring cancels out.

  python3 tools/ab.py --variants 0:0,128:0,64:0 [--stages 3] [--config c2]

Each variant is knobs:nt (aqz_stage_set_tuning).  For every stage, every
round runs each variant `reps` launches; prints min ms per (stage, variant).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))

import aqz  # noqa: E402
import torch  # noqa: E402

SPACE, TIME = 0, 2
CONFIGS = {
    # name: (dtype code, bytes per px, H, W, chunk, t-chunk, levels, frames/launch)
    "c2": (1, 2, 2048, 2048, 256, 64, 5, 64),
    "c1": (1, 2, 512, 512, 128, 64, 3, 64),
    "c3": (0, 1, 4096, 4096, 128, 32, 6, 32),
    "c5": (8, 4, 8192, 8192, 128, 4, 7, 4),
    "c4": (1, 2, 2048, 2048, 256, 64, 4, 64),  # + z: 256 planes, z-chunk 64
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0:0,128:0")
    ap.add_argument("--stages", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--config", default="c2")
    args = ap.parse_args()
    dt, bpp, H, W, ch, tch, levels, B = CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    fbytes = H * W * bpp
    nring = max(4, (2 << 30) // (B * fbytes))
    ring = torch.empty(nring * B * fbytes, dtype=torch.uint8, device=dev)
    ring.view(torch.int16).random_(0, 4096)
    dims = [(TIME, 0, tch, 1), (SPACE, H, ch, 1), (SPACE, W, ch, 1)]
    if args.config == "c4":
        dims = [(TIME, 0, 1, 1), (SPACE, 256, 64, 1), (SPACE, H, ch, 1), (SPACE, W, ch, 1)]
        levels = 0
    variants = [tuple(int(x) for x in v.split(":")) for v in args.variants.split(",")]
    stages = []
    for _ in range(args.stages):
        st = aqz.Stage(dims, dt, 1, max_batch_frames=B, layer_slots=2, force_levels=levels)
        print("levels", st.n_levels(), file=sys.stderr)
        st.set_stream(stream.cuda_stream)
        stages.append(st)
    state = {"i": 0}

    def launch(st):
        i = state["i"] = (state["i"] + 1) % nring
        st.append_ptr(ring.data_ptr() + i * B * fbytes, B)

    res = {}
    for _ in range(args.rounds):
        for si, st in enumerate(stages):
            for v in variants:
                st.set_tuning(*v)
                launch(st)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(stream)
                for _ in range(args.reps):
                    launch(st)
                e.record(stream)
                torch.cuda.synchronize()
                ms = s.elapsed_time(e) / args.reps
                res.setdefault((si, v), []).append(ms)
    hdr = "stage " + " ".join(f"{'k%d/nt%d' % v:>12s}" for v in variants)
    print(f"{args.config}: {B} frames of {H}x{W}x{bpp}B per launch, {levels} levels")
    print(hdr)
    for si in range(len(stages)):
        print(f"{si:5d} " + " ".join(f"{min(res[(si, v)]):12.4f}" for v in variants))
    for st in stages:
        st.close()


if __name__ == "__main__":
    main()
