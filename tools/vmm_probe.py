#!/usr/bin/env python3
"""Dev probe (not product): chunk-layer rings from the HIP virtual-memory
API (bench option ring_malloc_flags = 0x100 | log2(piece / granularity) << 9:
hipMemCreate pieces mapped into one reserved range), no placement search.
Prints creation time and the C2 launch time, step by step (flushes), so a
slow step shows where it is."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))

import aqz  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", type=int, required=True)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--arena", type=int, default=0,
                    help="ring_arena_bytes: every ring packed into one allocation")
    args = ap.parse_args()
    c = bench.CONFIGS[args.config]
    B = c["batch"]
    fbytes = c["dims"][-2][1] * c["dims"][-1][1] * bench.BPP[c["dtype"]]
    src = torch.empty(B * fbytes, dtype=torch.uint8, device="cuda")
    bench.fill_ring(torch, src, c["dtype"], 5)
    torch.cuda.synchronize()
    print(f"flags {args.flags:#x} arena {args.arena}: creating", flush=True)
    t = time.perf_counter()
    st = aqz.Stage(c["dims"], c["dtype"], c["method"], max_batch_frames=B,
                   layer_slots=bench.layer_slots_for(c, B), force_levels=c["force_levels"],
                   ring_malloc_flags=args.flags, ring_arena_bytes=args.arena)
    print(f"  created in {time.perf_counter() - t:.2f} s", flush=True)
    t = time.perf_counter()
    st.append_ptr(src.data_ptr(), B)
    st.synchronize()
    print(f"  first launch {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
    st.timing_mark(0)
    for _ in range(args.launches):
        st.append_ptr(src.data_ptr(), B)
    st.timing_mark(1)
    print(f"  {st.timing_elapsed() / args.launches:.4f} ms/launch", flush=True)
    st.close()


if __name__ == "__main__":
    main()
