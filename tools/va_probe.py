#!/usr/bin/env python3
# HISTORICAL (rounds 2-3): the AQZ_* environment switches this probe sets were
# removed in round 4 (kernel tuning is only in aqz_stage_bench_options, e.g.
# aqz.Stage(..., knobs=..., chunk_pad_bytes=...)); kept for the provenance of
# the profiles/ files it produced.
"""Dev probe (not product): does the stage's slow/fast mode follow the
virtual addresses of its chunk-layer rings?  Creates stages one after the
other with placement calibration off (AQZ_PLACEMENT_TRIES=1), shifting the
allocator between them with pads of varying size, and prints each stage's
ms per launch next to its large allocations (AQZ_DEBUG_ALLOC=1 lines)."""
import os
import sys

os.environ["AQZ_PLACEMENT_TRIES"] = "1"
os.environ["AQZ_DEBUG_ALLOC"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))

import aqz  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    c = bench.CONFIGS[cfg]
    B = c["batch"]
    h, w = c["dims"][-2][1], c["dims"][-1][1]
    fbytes = h * w * {0: 1, 1: 2, 8: 4}[c["dtype"]]
    src = torch.empty(2 * B * fbytes, dtype=torch.uint8, device="cuda")
    src.view(torch.int16).random_(-32768, 32767)
    print(f"src {src.data_ptr():#x}", flush=True)
    pads = []
    for i in range(n):
        pads.append(torch.empty((i % 5) * (48 << 20) + (1 << 20), dtype=torch.uint8,
                                device="cuda"))
        sys.stderr.flush()
        print(f"--- stage {i}", flush=True)
        st = aqz.Stage(c["dims"], c["dtype"], c["method"], max_batch_frames=B, layer_slots=2,
                       force_levels=c["force_levels"])
        best = 1e9
        for rnd in range(2):
            for k in range(2):
                st.append_ptr(src.data_ptr() + (k % 2) * B * fbytes, B)
            st.synchronize()
            st.timing_mark(0)
            for k in range(20):
                st.append_ptr(src.data_ptr() + (k % 2) * B * fbytes, B)
            st.timing_mark(1)
            best = min(best, st.timing_elapsed() / 20)
        sys.stderr.flush()
        print(f"stage {i} ms {best:.4f}", flush=True)
        st.close()


if __name__ == "__main__":
    main()
