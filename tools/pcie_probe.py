#!/usr/bin/env python3
"""PCIe probe: H2D alone, D2H alone, and both at once on two streams (the
ceilings of the end-to-end path; DESIGN.md 'End to end').  Buffers are
hipHostMalloc'd (aqz.HostBuffer, as the stage uses) and torch-pinned; copies
go through hipMemcpyAsync of the process's one HIP runtime."""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "acquire-zarr_amd"))
import aqz  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.init()
    aqz.lib()
    hip = C.CDLL("libamdhip64.so.7", mode=C.RTLD_GLOBAL)
    hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    hip.hipMemcpyAsync.restype = C.c_int
    n = 512 << 20
    reps = 5
    d_a = torch.empty(n, dtype=torch.uint8, device=dev)
    d_b = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    out = {"bytes": n}

    def timed(fn):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / reps

    for kind in ("hipHostMalloc", "torch_pinned"):
        if kind == "hipHostMalloc":
            hs, hd = aqz.HostBuffer(n), aqz.HostBuffer(n)
            src, dst = hs.ptr, hd.ptr
        else:
            hs = torch.empty(n, dtype=torch.uint8).pin_memory()
            hd = torch.empty(n, dtype=torch.uint8).pin_memory()
            src, dst = hs.data_ptr(), hd.data_ptr()

        def h2d():
            assert hip.hipMemcpyAsync(d_a.data_ptr(), src, n, 1, s1.cuda_stream) == 0

        def d2h():
            assert hip.hipMemcpyAsync(dst, d_b.data_ptr(), n, 2, s2.cuda_stream) == 0

        def both():
            h2d()
            d2h()

        def both_rev():
            d2h()
            h2d()

        def pieces(mb, interleave):
            p = mb << 20

            def fn():
                if interleave:
                    for o in range(0, n, p):
                        assert hip.hipMemcpyAsync(d_a.data_ptr() + o, src + o, p, 1,
                                                  s1.cuda_stream) == 0
                        assert hip.hipMemcpyAsync(dst + o, d_b.data_ptr() + o, p, 2,
                                                  s2.cuda_stream) == 0
                else:  # all H2D pieces issued first, then all D2H pieces
                    for o in range(0, n, p):
                        assert hip.hipMemcpyAsync(d_a.data_ptr() + o, src + o, p, 1,
                                                  s1.cuda_stream) == 0
                    for o in range(0, n, p):
                        assert hip.hipMemcpyAsync(dst + o, d_b.data_ptr() + o, p, 2,
                                                  s2.cuda_stream) == 0
            return fn

        t_h, t_d = timed(h2d), timed(d2h)
        t_b, t_r = timed(both), timed(both_rev)
        out[kind] = {"h2d_gbs": round(n / t_h / 1e9, 2), "d2h_gbs": round(n / t_d / 1e9, 2),
                     "duplex_total_gbs": round(2 * n / t_b / 1e9, 2),
                     "duplex_rev_total_gbs": round(2 * n / t_r / 1e9, 2)}
        for mb in (8, 32, 64, 128):
            for il in (True, False):
                t = timed(pieces(mb, il))
                out[kind][f"pieces{mb}MiB_{'interleaved' if il else 'h2d_first'}_total_gbs"] = \
                    round(2 * n / t / 1e9, 2)

    print(json.dumps(out))


if __name__ == "__main__":
    main()
