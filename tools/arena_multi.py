#!/usr/bin/env python3
"""Dev probe (not product): do successive ring arenas (the shipped 2 MiB
virtual-memory pieces) of one process land in different placement bands?
Creates `stages` C2 stages one after another, every earlier one still held,
and times each on the same source; then the HBM probe of the copy + 1/3
shape for reference."""
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
    ap.add_argument("--stages", type=int, default=4)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--launches", type=int, default=30)
    args = ap.parse_args()
    c = bench.CONFIGS[args.config]
    B = c["batch"]
    fbytes = c["dims"][-2][1] * c["dims"][-1][1] * bench.BPP[c["dtype"]]
    src = torch.empty(B * fbytes, dtype=torch.uint8, device="cuda")
    bench.fill_ring(torch, src, c["dtype"], 5)
    torch.cuda.synchronize()
    held, out = [], []
    for s in range(args.stages):
        st = aqz.Stage(c["dims"], c["dtype"], c["method"], max_batch_frames=B,
                       layer_slots=bench.layer_slots_for(c, B), force_levels=c["force_levels"],
                       ring_malloc_flags=args.flags)
        for _ in range(2):
            st.append_ptr(src.data_ptr(), B)
        st.synchronize()
        st.timing_mark(0)
        for _ in range(args.launches):
            st.append_ptr(src.data_ptr(), B)
        st.timing_mark(1)
        out.append(round(st.timing_elapsed() / args.launches, 4))
        held.append(st)
    probe = bench.hbm_probe(aqz, 0)["copy_third_bus_gbs"]
    print(f"{args.config} flags {args.flags:#x}: stages {out} probe copy+1/3 {probe} GB/s",
          flush=True)
    for st in held:
        st.close()


if __name__ == "__main__":
    main()
