"""Which allocation decides a C2 stage's placement band?

One C2 stage (bench geometry, no placement search) and one 2 GiB device
source ring.  Between timed blocks of launches, fresh chunk-layer rings are
allocated for a set of levels (aqz_stage_bench_replace_rings; the old rings
stay allocated, so the new ones land in other memory), or a fresh source
ring.  If a band moves only when level 0's ring moves, level 0's placement
decides it; and so on.  One JSON line per block to stdout.

  python3 tools/placement_localize.py [--trials 6] [--launches 40]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=6)
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--ring-flags", type=int, default=0,
                    help="hipExtMallocWithFlags flags of the rings (4: contiguous)")
    ap.add_argument("--spacer-gib", type=float, default=0.0,
                    help="ring_spacer_bytes: allocated before the rings, freed after")
    ap.add_argument("--plan", default="",
                    help="comma list of steps: pre=MiB (a held torch allocation made "
                         "before the stage), start, src (fresh source ring), "
                         "L=mask (fresh rings for those levels), all")
    args = ap.parse_args()
    import torch
    import aqz
    import bench
    cfg = bench.CONFIGS["c2"]
    B = args.batch
    steps = args.plan.split(",") if args.plan else []
    held = []
    while steps and steps[0].startswith("pre="):
        held.append(torch.empty(int(steps.pop(0)[4:]) << 20, dtype=torch.uint8,
                                device="cuda"))
    st = aqz.Stage(cfg["dims"], cfg["dtype"], cfg["method"], force_levels=5,
                   max_batch_frames=B, layer_slots=bench.layer_slots_for(cfg, B),
                   ring_malloc_flags=args.ring_flags,
                   ring_spacer_bytes=int(args.spacer_gib * (1 << 30)))
    fbytes = 2048 * 2048 * 2
    nb = 256 // B if B <= 256 else 1
    srcs = []

    def new_source(seed):
        r = torch.empty(256 * fbytes, dtype=torch.uint8, device="cuda")
        bench.fill_ring(torch, r, cfg["dtype"], seed)
        torch.cuda.synchronize()
        srcs.append(r)
        return r.data_ptr()

    base = new_source(1)

    def timed(tag):
        for s in range(3):
            st.append_ptr(base + (s % nb) * B * fbytes, B)
        st.synchronize()
        st.timing_mark(0)
        for s in range(args.launches):
            st.append_ptr(base + (s % nb) * B * fbytes, B)
        st.timing_mark(1)
        st.synchronize()
        return st.timing_elapsed() / args.launches

    nl = st.n_levels()
    if not steps:
        steps = ["start"] + ["L=1"] * args.trials + [f"L={((1 << nl) - 1) & ~1}"] * \
            args.trials + ["src"] * args.trials + ["all"] * args.trials
    out = []
    t0 = time.time()
    for step in steps:
        if step == "src":
            base = new_source(100 + len(srcs))
        elif step == "all":
            st.replace_rings((1 << nl) - 1)
        elif step.startswith("L="):
            st.replace_rings(int(step[2:], 0))
        ms, ms2 = timed(step), timed(step)
        out.append([step, round(ms, 4), round(ms2, 4)])
    st.close()
    print(json.dumps({"plan": args.plan, "ring_flags": args.ring_flags,
                      "spacer_gib": args.spacer_gib, "summary": out,
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
