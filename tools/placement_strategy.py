#!/usr/bin/env python3
"""Dev probe (not product): placement-search strategies side by side.  One
stage at a time (created, measured, destroyed): no search, mode 0 (free the
loser + a spacer) and mode 1 (hold every candidate), cycling for `rounds`.
Per stage it prints the search's candidates, the kept candidate's time, its
re-time alone (kept_ms_final), the creation peak vs the bench estimate,
and the steady state: `steps` launches from a random 2 GiB source ring as
bench.py times them."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))

import aqz  # noqa: E402
import torch  # noqa: E402

SPACE, TIME = 0, 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tries", type=int, default=16)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--spacer-mb", type=int, default=128)
    ap.add_argument("--modes", default="off,0,1")
    args = ap.parse_args()
    B, H, W = 128, 2048, 2048
    fbytes = H * W * 2
    dev = torch.device("cuda", 0)
    src = torch.empty(2 * B * fbytes, dtype=torch.uint8, device=dev)
    src.view(torch.int16).random_(-32768, 32767)
    dims = [(TIME, 0, 64, 1), (SPACE, H, 256, 1), (SPACE, W, 256, 1)]
    for rnd in range(args.rounds):
        for mode in args.modes.split(","):
            kw = dict(max_batch_frames=B, layer_slots=2, force_levels=5)
            if mode != "off":
                kw.update(placement_tries=args.tries, placement_mode=int(mode),
                          placement_spacer_bytes=args.spacer_mb << 20)
            est = aqz.estimate_memory(dims, 1, 1, **kw)
            st = aqz.Stage(dims, 1, 1, **kw)
            pl = st.placement()
            st.append_ptr(src.data_ptr(), B)
            st.synchronize()
            st.timing_mark(0)
            for k in range(args.steps):
                st.append_ptr(src.data_ptr() + (k % 2) * B * fbytes, B)
            st.timing_mark(1)
            steady = st.timing_elapsed() / args.steps
            kept = pl["candidates_ms"][pl["kept"]] if pl["candidates_ms"] else None
            rec = {"round": rnd, "mode": mode, "steady_ms": round(steady, 5),
                   "kept_ms": kept, "kept_ms_final": pl["kept_ms_final"],
                   "n": len(pl["candidates_ms"]), "candidates": pl["candidates_ms"],
                   "peak_gib": round(pl["peak_device_bytes"] / 2**30, 3),
                   "usage_gib": round(st.memory_usage()["device_bytes"] / 2**30, 3),
                   "estimate_gib": round(est["device_bytes"] / 2**30, 3)}
            print(json.dumps(rec), flush=True)
            st.close()
            del st
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
