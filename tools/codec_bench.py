#!/usr/bin/env python3
"""Dev harness (not product): device compressor throughput (blosc-lz4,
blosc-zstd or plain zstd) on a C2 level-0 chunk layer (64 chunks of
256x256x64 u16 = 8 MiB) for several payloads, next to c-blosc 1.21.0 /
libzstd (clevel 5, one thread) on the host.

  python3 tools/codec_bench.py [--reps 5] [--shuffle 1] [--codec lz4|blosc-zstd|zstd]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import aqz  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402


def payload(kind, n_chunks, chunk_bytes, dev):
    n_px = n_chunks * chunk_bytes // 2
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    if kind == "camera":
        x = torch.arange(n_px, device=dev, dtype=torch.float32)
        v = 1000.0 + 200.0 * torch.sin(x / 977.0) + 30.0 * torch.randn(n_px, device=dev, generator=g)
        return v.clamp(0, 65535).to(torch.int32).to(torch.int16).view(torch.uint8)
    if kind == "dim":   # low-light sCMOS: offset 100, a few counts of noise
        v = 100.0 + 3.0 * torch.randn(n_px, device=dev, generator=g)
        return v.clamp(0, 65535).to(torch.int32).to(torch.int16).view(torch.uint8)
    if kind == "zeros":
        return torch.zeros(n_chunks * chunk_bytes, dtype=torch.uint8, device=dev)
    return torch.randint(0, 256, (n_chunks * chunk_bytes,), dtype=torch.uint8, device=dev,
                         generator=g)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shuffle", type=int, default=1)
    ap.add_argument("--clevel", type=int, default=5)
    ap.add_argument("--kinds", default="camera,dim,zeros,random")
    ap.add_argument("--codec", default="lz4", choices=["lz4", "blosc-zstd", "zstd"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n_chunks, cb = 64, 256 * 256 * 64 * 2
    codec = {"lz4": 1, "blosc-zstd": 2, "zstd": 3}[args.codec]
    comp = aqz.Compressor(cb, 2, codec=codec, clevel=args.clevel, shuffle=args.shuffle)
    cap = comp.max_bytes(n_chunks)
    dst = torch.empty(cap, dtype=torch.uint8, device=dev)
    off = torch.empty(n_chunks + 1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()
    try:
        from codec_helpers import libblosc, libblosc_compress, zstd_compress
        have_blosc = libblosc() is not None
    except Exception:
        have_blosc = False
    print(f"layer: {n_chunks} chunks x {cb >> 20} MiB u16, {args.codec}, shuffle {args.shuffle}, "
          f"blocksize {comp.blocksize}")
    for kind in args.kinds.split(","):
        src = payload(kind, n_chunks, cb, dev)
        run = lambda: comp.run_ptr(src.data_ptr(), cb, n_chunks, dst.data_ptr(), cap,
                                   off.data_ptr(), stream.cuda_stream)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        total = int(off[-1].item())
        line = (f"{kind:7s} device {ms:8.3f} ms/layer  {n_chunks * cb / ms / 1e6:8.1f} GB/s in  "
                f"ratio {n_chunks * cb / total:6.3f}")
        if have_blosc:
            chunk = src[:cb].cpu().numpy().tobytes()
            t0 = time.perf_counter()
            if codec == 3:
                fr = zstd_compress(chunk, args.clevel)
            else:
                fr = libblosc_compress(chunk, 2, args.clevel, args.shuffle,
                                       b"zstd" if codec == 2 else b"lz4")
            dt = time.perf_counter() - t0
            line += f"   | host 1 thread {cb / dt / 1e9:6.2f} GB/s ratio {cb / len(fr):6.3f}"
        print(line, flush=True)
    comp.close()


if __name__ == "__main__":
    main()
