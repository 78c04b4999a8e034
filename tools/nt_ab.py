#!/usr/bin/env python3
"""Dev probe (not product): nontemporal load/store A/B on the SAME stage
(same placement), via aqz_stage_set_tuning(knobs=0, nt) -- nt bit 1 = input
loads, bit 2 = level-0 tile stores, bit 4 = level-1/2 stores.  For the full
C2 stage and the pyramid-only stage, several stage instances each.  Prints
ms per 128-frame launch."""
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
    ap.add_argument("--instances", type=int, default=3)
    ap.add_argument("--nt", default="0,1,2,3,4,5,6,7")
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()
    B, H, W = 128, 2048, 2048
    fbytes = H * W * 2
    src = torch.empty(2 * B * fbytes, dtype=torch.uint8, device="cuda")
    src.view(torch.int16).random_(-32768, 32767)
    dims = [(TIME, 0, 64, 1), (SPACE, H, 256, 1), (SPACE, W, 256, 1)]
    nts = [int(x) for x in args.nt.split(",")]
    for pyr in (False, True):
        for inst in range(args.instances):
            st = aqz.Stage(dims, 1, 1, max_batch_frames=B, layer_slots=2, force_levels=5,
                           skip_level0_split=pyr)
            row = []
            for rnd in range(2):
                for j, nt in enumerate(nts):
                    st.set_tuning(0, nt)
                    for k in range(2):
                        st.append_ptr(src.data_ptr() + (k % 2) * B * fbytes, B)
                    st.synchronize()
                    st.timing_mark(0)
                    for k in range(args.reps):
                        st.append_ptr(src.data_ptr() + (k % 2) * B * fbytes, B)
                    st.timing_mark(1)
                    ms = st.timing_elapsed() / args.reps
                    if rnd == 0:
                        row.append(ms)
                    else:
                        row[j] = min(row[j], ms)
            name = "pyr " if pyr else "full"
            print(f"{name} inst{inst} " + " ".join(f"nt{nt}={v:.4f}" for nt, v in zip(nts, row)),
                  flush=True)
            st.close()


if __name__ == "__main__":
    main()
