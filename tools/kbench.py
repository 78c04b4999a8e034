#!/usr/bin/env python3
# HISTORICAL (rounds 2-3): the AQZ_* environment switches this probe sets were
# removed in round 4 (kernel tuning is only in aqz_stage_bench_options, e.g.
# aqz.Stage(..., knobs=..., chunk_pad_bytes=...)); kept for the provenance of
# the profiles/ files it produced.
"""Dev harness: time stage variants and copy baselines in ONE process
(interleaved rounds), print a table.  Not part of the product or the bench
contract."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))

import aqz  # noqa: E402
import torch  # noqa: E402

SPACE, TIME = 0, 2


def timed(fn, reps, stream):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record(stream)
    for _ in range(reps):
        fn()
    e.record(stream)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--bpc", type=int, default=0)
    ap.add_argument("--rh", default="6,7")
    ap.add_argument("--bpcs", default="")
    ap.add_argument("--knobs", default="")
    ap.add_argument("--depth", action="store_true")
    ap.add_argument("--nt", default="0")
    ap.add_argument("--pads", default="")
    ap.add_argument("--full4", action="store_true")
    ap.add_argument("--prealloc-gb", type=float, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    B, H, W = 64, 2048, 2048
    fbytes = H * W * 2
    ring = torch.empty(4 * B * fbytes, dtype=torch.uint8, device=dev)
    print(f"ring {ring.data_ptr():#x}", file=sys.stderr)
    ring.view(torch.int16).random_(-32768, 32767)
    dst = torch.empty(B * fbytes, dtype=torch.uint8, device=dev)
    hold = torch.empty(int(args.prealloc_gb * 2**30), dtype=torch.uint8, device=dev) if args.prealloc_gb else None
    dims = [(TIME, 0, 64, 1), (SPACE, H, 256, 1), (SPACE, W, 256, 1)]
    variants = {}
    bytes_moved_extra = {}

    def mk(name, **kw):
        print(f"stage {name}", file=sys.stderr)
        st = aqz.Stage(dims, 1, 1, max_batch_frames=B, layer_slots=2, **kw)
        st.set_stream(stream.cuda_stream)
        variants[name] = st

    for rh in args.rh.split(","):
        os.environ["AQZ_REGION_ROWS_LOG2"] = rh
        for j, nt in enumerate(args.nt.split(",")):
            os.environ["AQZ_NT"] = nt
            mk(f"full5_rh{rh}_nt{nt}_{j}", force_levels=5)
        os.environ["AQZ_NT"] = "0"
        mk(f"pyr5_rh{rh}", force_levels=5, skip_level0_split=True)
    os.environ.pop("AQZ_REGION_ROWS_LOG2")
    os.environ.pop("AQZ_NT")
    for j, kn in enumerate(args.knobs.split(",")):
        if kn:
            os.environ["AQZ_KNOBS"] = kn
            mk(f"full5_k{kn}_{j}", force_levels=5)
            bytes_moved_extra[f"full5_k{kn}_{j}"] = B * fbytes * (2 + (1 / 4 + 1 / 16 + 1 / 64 + 1 / 256))
            if args.full4:
                mk(f"full4_k{kn}_{j}", force_levels=4)
                bytes_moved_extra[f"full4_k{kn}_{j}"] = B * fbytes * (2 + (1 / 4 + 1 / 16 + 1 / 64))
            os.environ.pop("AQZ_KNOBS")
    for j, pad in enumerate(args.pads.split(",")):
        if pad:
            os.environ["AQZ_CHUNK_PAD"] = pad
            mk(f"full5_pad{pad}_{j}", force_levels=5)
            bytes_moved_extra[f"full5_pad{pad}_{j}"] = B * fbytes * (2 + (1 / 4 + 1 / 16 + 1 / 64 + 1 / 256))
            os.environ.pop("AQZ_CHUNK_PAD")
    mk("split_only", multiscale=False)
    for nl in ((2, 3, 4) if args.depth else ()):
        mk(f"pyr{nl}_only", force_levels=nl, skip_level0_split=True)
        bytes_moved_extra[f"pyr{nl}_only"] = B * fbytes * (1 + sum(4.0 ** -k for k in range(1, nl)))
        mk(f"full{nl}", force_levels=nl)
        bytes_moved_extra[f"full{nl}"] = B * fbytes * (2 + sum(4.0 ** -k for k in range(1, nl)))
    mk("full4_refrule")
    state = {"i": 0}

    def run_stage(st):
        def f():
            i = state["i"] = (state["i"] + 1) % 4
            st.append_ptr(ring.data_ptr() + i * B * fbytes, B)
        return f

    def copy():
        i = state["i"] = (state["i"] + 1) % 4
        dst.copy_(ring[i * B * fbytes:(i + 1) * B * fbytes])

    def read_only():
        i = state["i"] = (state["i"] + 1) % 4
        return ring[i * B * fbytes:(i + 1) * B * fbytes].view(torch.int64).sum()

    bytes_moved = {
        **{f"full5_rh{rh}_nt{nt}_{j}": B * fbytes * (2 + (1 / 4 + 1 / 16 + 1 / 64 + 1 / 256)) for rh in args.rh.split(",") for j, nt in enumerate(args.nt.split(","))},
        **{f"pyr5_rh{rh}": B * fbytes * (1 + (1 / 4 + 1 / 16 + 1 / 64 + 1 / 256)) for rh in args.rh.split(",")},
        "split_only": B * fbytes * 2,
        "full4_refrule": B * fbytes * (2 + (1 / 4 + 1 / 16 + 1 / 64)),
        "torch_copy": B * fbytes * 2,
        "torch_sum": B * fbytes,
        **bytes_moved_extra,
    }
    res = {k: [] for k in bytes_moved}
    for rnd in range(args.rounds):
        for name, st in variants.items():
            res[name].append(timed(run_stage(st), args.reps, stream))
        res["torch_copy"].append(timed(copy, args.reps, stream))
        res["torch_sum"].append(timed(read_only, args.reps, stream))
    print(f"{'variant':16s} {'ms/64fr':>9s} {'in GB/s':>9s} {'bus GB/s':>9s}")
    for k, v in res.items():
        ms = min(v)
        print(f"{k:20s} {ms:9.4f} {B * fbytes / ms / 1e6:9.1f} {bytes_moved[k] / ms / 1e6:9.1f}")
    for st in variants.values():
        st.close()


if __name__ == "__main__":
    main()
