#!/usr/bin/env python3
"""Dev probe (not product): what differs between a slow-band and a fast-band
placement in the memory pipeline's request mix?  Stage A keeps its first
allocation (placement_tries 0: the slow band on every box so far), stage B
searches (16 tries).  Each then runs 2 + 20 launches of C2 on the same
source.  Run it under `rocprofv3 --pmc ...`; the first 22 dispatches of the
strip kernel are stage A's, the last 22 stage B's (B's search launches sit
in between).  With --summarise DIR it reads those counter CSVs instead.

Counter sets (one rocprofv3 pass each): the TCP->TCC request types by
memory type (RW / NC / CC / UC, reads then writes) and the TCP->TCC request
latencies."""
import argparse
import csv
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))
    import aqz
    import torch
    import bench
    c = bench.CONFIGS["c2"]
    B = c["batch"]
    fbytes = c["dims"][-2][1] * c["dims"][-1][1] * 2
    src = torch.empty(B * fbytes, dtype=torch.uint8, device="cuda")
    bench.fill_ring(torch, src, c["dtype"], 5)
    torch.cuda.synchronize()
    out = []
    for name, tries in (("A", 0), ("B", 16)):
        st = aqz.Stage(c["dims"], c["dtype"], c["method"], max_batch_frames=B,
                       layer_slots=bench.layer_slots_for(c, B),
                       force_levels=c["force_levels"], placement_tries=tries)
        for _ in range(2):
            st.append_ptr(src.data_ptr(), B)
        st.synchronize()
        st.timing_mark(0)
        for _ in range(20):
            st.append_ptr(src.data_ptr(), B)
        st.timing_mark(1)
        out.append((name, st.timing_elapsed() / 20, st.placement().get("candidates_ms")))
        if name == "A":
            keep = st  # held: B's allocations come after A's
        else:
            st.close()
    keep.close()
    for name, ms, cand in out:
        print(f"stage {name}: {ms:.4f} ms/launch  candidates {cand}", flush=True)


def summarise(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "fused_pyramid_strip" in r.get("Kernel_Name", ""):
                    rows.append(r)
    by = {}
    for r in rows:
        key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
        by.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(by)
    if len(ids) < 44:
        print("too few dispatches", len(ids))
        return
    for name, sel in (("A", ids[2:22]), ("B", ids[-20:])):
        names = sorted({k for i in sel for k in by[i]})
        vals = {k: sum(by[i].get(k, 0.0) for i in sel) / len(sel) for k in names}
        print(name, " ".join(f"{k}={v:.4g}" for k, v in vals.items()))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--summarise", default=None)
    a = ap.parse_args()
    if a.summarise:
        summarise(a.summarise)
    else:
        run(a)
