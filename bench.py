#!/usr/bin/env python3
"""Benchmark: input GB/s of the device-resident multiscale stage.

One "step" = one launch batch of frames through the whole hot path of
MultiscaleArray::write_frame: level-0 chunk-tile split + pyramid + tile split
of every level into device-resident chunk layers (+ has_data flags).  Frames
are synthetic, already resident in HBM (a >= 2 GiB ring, well past the 256 MiB
Infinity Cache).  With --gpus N (torch.distributed.run, one rank per GPU)
every rank runs its own independent stream (weak scaling, no collective on
the data path; only the barrier and the max-over-ranks of the timed region).

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement".
"""
import argparse
import ctypes as C
import json
import os
import resource
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

SPACE, CHANNEL, TIME = 0, 1, 2
U8, U16, F32 = 0, 1, 8
DECIMATE = 0
MEAN = 1
BPP = {U8: 1, U16: 2, F32: 4}

# aqz_stage_options.placement_tries, as the binding passes it: the shipped
# rings (one arena of 2 MiB virtual-memory pieces) are
# timed at creation against a streaming probe of the same memory; only when
# they run more than 3% over that expectation does one fresh arena follow
# (roofline.placement: candidates, expectation, the one kept).
PLACEMENT = dict(placement_tries=2)

DTYPE_WORDS = {U8: "uint8", U16: "uint16", F32: "float32"}

CONFIGS = {
    # BASELINE.json configs[0], the reference's CPU-runnable case (SURVEY
    # §8a: u16 512x512, 3 levels at 128-px chunks, decimate), device-resident;
    # 2048-frame launches (1 GiB of input): 2-8% faster than 1024 on the same
    # stages (profiles/r05_c1_launch_ab.txt)
    "c1": dict(workload="uint16 512x512 frames, 3-level pyramid (512..128 px), 128x128 "
                        "chunks (t-chunk 64), decimate, device-resident",
               dims=[(TIME, 0, 64, 1), (SPACE, 512, 128, 1), (SPACE, 512, 128, 1)],
               dtype=U16, method=DECIMATE, force_levels=0, batch=2048, ring=4096),
    # BASELINE.json configs[1] -- the metric's config.  The reference level
    # rule (downsampler.cpp:512-541) stops at 4 levels for 256-px chunks;
    # force_levels keeps halving to the requested 5 (L4 = 128 px, one
    # partial 256x256 chunk), pixel values unchanged.
    # 512-frame launches (4 GiB of input): a launch's ramp-up and drain cost
    # ~15 us whatever its size; 2.3-3.1% faster than 256 on the same stage,
    # 1024 adds 0.5% more (profiles/r05_launch_size_ab.txt)
    "c2": dict(workload="uint16 2048x2048 frames, 5-level pyramid (2048..128 px), "
                        "256x256 chunks (t-chunk 64), mean, level-0 split + pyramid + "
                        "tile split of all levels, device-resident",
               dims=[(TIME, 0, 64, 1), (SPACE, 2048, 256, 1), (SPACE, 2048, 256, 1)],
               dtype=U16, method=MEAN, force_levels=5, batch=512, ring=512),
    # same, reference level rule (4 levels)
    "c2-ref4": dict(workload="uint16 2048x2048 frames, 4-level pyramid (reference rule "
                             "at 256-px chunks), t-chunk 64, mean, device-resident",
                    dims=[(TIME, 0, 64, 1), (SPACE, 2048, 256, 1), (SPACE, 2048, 256, 1)],
                    dtype=U16, method=MEAN, force_levels=0, batch=512, ring=512),
    # 256-frame launches (4 GiB of input): 128 was 4.7% faster than 64
    # (profiles/r05_c3_launch_ab.txt), 256 1.6-2.4% faster than 128 on the
    # same stage (profiles/r05_launch_size_ab.txt)
    "c3": dict(workload="uint8 4096x4096 frames, 6-level pyramid, 128x128 chunks, mean, "
                        "device-resident",
               dims=[(TIME, 0, 32, 1), (SPACE, 4096, 128, 1), (SPACE, 4096, 128, 1)],
               dtype=U8, method=MEAN, force_levels=0, batch=256, ring=256),
    # BASELINE configs[3]: a 256-plane volume, 2x2x2 pyramid (z 256->128->
    # 64->64, xy 2048->1024->512->256), one volume per launch (1.7-7% faster
    # than half a volume on the same stage).  With --gpus N rank r owns z slab
    # [lo, hi) of every volume of the stream (aqz_stage_options z_slab_*,
    # slabs aligned to the 4-plane z groups): its stage receives only those
    # planes, and frame ids skip the other ranks' planes.
    "c4": dict(workload="uint16 2048x2048x256 light-sheet volume, 4-level 3-D (2x2x2) "
                        "pyramid, 256x256x64 chunks, mean, device-resident",
               dims=[(TIME, 0, 1, 1), (SPACE, 256, 64, 1), (SPACE, 2048, 256, 1),
                     (SPACE, 2048, 256, 1)],
               dtype=U16, method=MEAN, force_levels=0, batch=256, ring=512),
    # 16-frame launches (4 GiB): 1.2-2.7% faster than 8 on the same stage
    "c5": dict(workload="float32 8192x8192 frames, 7-level pyramid, 128x128 chunks, mean, "
                        "device-resident (one camera stream per GPU)",
               dims=[(TIME, 0, 4, 1), (SPACE, 8192, 128, 1), (SPACE, 8192, 128, 1)],
               dtype=F32, method=MEAN, force_levels=0, batch=16, ring=16),
}


def layer_slots_for(cfg, B):
    """Chunk-layer ring slots of the device-resident run: a 2-D launch of B
    frames spans B / t-chunk layers of every level, which the ring must hold
    (at least 2)."""
    if len(cfg["dims"]) != 3:
        return 2
    return max(2, -(-B // cfg["dims"][0][2]))


def hbm_probe(aqz, device):
    """Live streaming probe of this device (aqz_probe_hbm): 512 MiB read per
    launch from a 2 GiB ring, 16-B nontemporal lane loads, 24 KiB per
    workgroup, the better of nontemporal and plain stores; GB/s of each
    access shape the stage runs."""
    out = {}
    for key, shape, wr in (("read_gbs", aqz.PROBE_READ, 0.0),
                           ("copy_bus_gbs", aqz.PROBE_COPY, 1.0),
                           ("copy_third_bus_gbs", aqz.PROBE_COPY_THIRD, 4.0 / 3.0),
                           ("read_third_bus_gbs", aqz.PROBE_READ_THIRD, 1.0 / 3.0)):
        flavours = (0,) if shape == aqz.PROBE_READ else (0, aqz.PROBE_PLAIN_STORES)
        runs = [aqz.probe_hbm(shape | f, 512 << 20, 20, device)
                for _ in range(2) for f in flavours]
        ms, rd = min(r[0] for r in runs), runs[0][1]
        out[key] = round(rd * (1 + wr) / (ms * 1e-3) / 1e9, 1)
        if shape == aqz.PROBE_READ_THIRD:
            out["read_third_input_gbs"] = round(rd / (ms * 1e-3) / 1e9, 1)
    out["read_frac_of_spec"] = round(out["read_gbs"] / HBM_PEAK_GBS, 4)
    out["source"] = "aqz_probe_hbm (include/aqz_gpu_bench.h), measured in this run"
    return out


def level_sizes(stage):
    out = []
    for l in range(stage.n_levels()):
        d = stage.level_dims(l)
        out.append((d[-2][1], d[-1][1]))
    return out


def fill_ring(torch, ring, dtype, seed):
    g = torch.Generator(device=ring.device)
    g.manual_seed(seed)
    if dtype == U16:
        ring.view(torch.int16).random_(-32768, 32767, generator=g)
    elif dtype == U8:
        ring.view(torch.uint8).random_(0, 256, generator=g)
    else:
        ring.view(torch.float32).uniform_(0.0, 65535.0, generator=g)


def device_code_sha256(path):
    """sha256 of a shared library's device code (its .hip_fatbin section:
    every gfx950 kernel code object), read from the ELF section table.  Two
    builds that differ only in host code have the same value, so a kernel
    profile of one describes the other's kernels."""
    import hashlib
    import struct
    try:
        with open(path, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    if data[:4] != b"\x7fELF" or data[4] != 2:  # ELF64 only
        return None
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def sec(i):
        name, _, _, _, off, size = struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)
        return name, off, size

    _, stroff, _ = sec(shstrndx)
    for i in range(shnum):
        name, off, size = sec(i)
        end = data.index(b"\0", stroff + name)
        if data[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(data[off:off + size]).hexdigest()
    return None


def lib_sha256():
    """sha256 of the libaqz_gpu.so this process loaded (aqz.lib())."""
    import hashlib
    import aqz
    try:
        with open(aqz.lib()._name, "rb") as fh:
            return hashlib.sha256(fh.read()).hexdigest()
    except (OSError, AttributeError):
        return None


def lib_device_code_sha256():
    """device_code_sha256 of the libaqz_gpu.so this process loaded."""
    import aqz
    try:
        return device_code_sha256(aqz.lib()._name)
    except AttributeError:
        return None


def pmc_traffic(config, pyramid_only, kernel, frames, ring_allocation, run_ms=None,
                lib_sha=None, dev_sha=None):
    """Per-launch HBM bytes of the dominant kernel from the newest committed
    rocprofv3 PMC summary for this configuration whose rings were allocated
    the same way as this run's (tools/profile.sh -> tools/pmc_summary.py ->
    profiles/<round>_<config>_pmc.json: FETCH_SIZE x2 + WRITE_SIZE, the
    gfx950 correction of MI355X_MICROARCH.md; the summary records the
    profiled bench line's ring_allocation).  PMC counters cannot be read
    inside a plain run, so the value is the profiled run of this same
    command; (None, None, None) when no summary matches."""
    import glob
    name = config + ("-pyr" if pyramid_only else "")
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_{name}_pmc.json")))
    found = []
    for f in files:
        d = json.load(open(f))
        if (d.get("config") == name and kernel and kernel in d.get("kernel", "")
                and d.get("ring_allocation") == ring_allocation):
            found.append((f, d))
    if not found:
        return None, None, None
    # a profile of the library build this run loaded, when there is one,
    # else of a build with the same device code (host-only changes)
    same = [fd for fd in found if lib_sha and fd[1].get("lib_sha256") == lib_sha]
    if not same and dev_sha:
        same = [fd for fd in found if fd[1].get("device_code_sha256") == dev_sha]
    found = same or found
    # MI355X boxes run the same kernel at different speeds (DESIGN.md
    # section 5); the bytes do not change with the box.  Of the profiles of
    # this configuration and ring allocation, the one whose kernel time is
    # closest to this run's represents it best (newest on a tie).
    def gap(fd):
        pa = fd[1].get("steady_avg_duration_ns") or fd[1].get("avg_duration_ns") or 0.0
        fpl = fd[1].get("frames_per_launch") or frames
        return abs(pa * 1e-6 * frames / fpl - run_ms) if run_ms else 0.0
    f, d = min(reversed(found), key=gap)
    # (traffic is linear in the frames of a launch: a profile of another
    # launch size is scaled to this one)
    t = d["traffic_bytes_per_launch"]
    fpl = d.get("frames_per_launch")
    if fpl and fpl != frames:
        t = int(round(t * frames / fpl))
    return t, os.path.relpath(f, REPO), d


def ring_allocation(pl):
    """How the chunk-layer rings were allocated (aqz_placement_report.mode)."""
    if pl.get("mode") == 3:
        return ("one arena of 2 MiB virtual-memory pieces" +
                (", fresh arena kept" if pl.get("kept") else ""))
    if pl.get("candidates_ms"):
        return "per-level allocations, placement search"
    return "per-level allocations (rings under 256 MiB), no search"


def cpu_baseline(cfg, seconds):
    """The reference's CPU path timed on this host's cores (rank 0 only):
    the compiled reference (oracle/_ref) when present, else the C port.
    Downsampler::add_frame runs on the one frame-consumer thread
    (zarr.stream.cpp:1683-1684); the reference's tile split is OpenMP over
    tiles (array.cpp:575), so its restated loop runs on OMP_NUM_THREADS."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_bindings as ob
    dims = list(cfg["dims"])
    dt, m = cfg["dtype"], cfg["method"]
    h, w = dims[-2][1], dims[-1][1]
    # The CPU reference cannot produce the forced 5th level at 256-px chunks;
    # its 5-level pyramid for these frames is the 128-px-chunk configuration
    # (identical pixels).
    if cfg.get("force_levels"):
        dims[-1] = (SPACE, w, 128, 1)
        dims[-2] = (SPACE, h, 128, 1)
    dims[0] = (TIME, 0, 1, 1)
    frames = ob.synthetic_frames(dt, 4, h, w, 99)
    kind = "reference" if ob.ref_available() else "port"
    ds = ob.OracleDownsampler(dims, dt, m, 0, use_ref=(kind == "reference"))
    L = ds.n_levels()
    ldims = [ds.level_dims(l) for l in range(L)]
    if kind == "reference":
        R = ob.ref()
        R.ref_split_create.argtypes = [C.POINTER(ob.Dim), C.c_int, C.c_int]
        R.ref_split_create.restype = C.c_void_p
        R.ref_split_write.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p]
        R.ref_split_write.restype = C.c_size_t
        R.ref_split_destroy.argtypes = [C.c_void_p]
        keep = [ob.dims_array(d) for d in ldims]
        sp = [R.ref_split_create(keep[l], len(ldims[l]), dt) for l in range(L)]

        def split(l, img):
            R.ref_split_write(sp[l], 0, img.ctypes.data)
    else:
        od = [ob.OracleDims(d, dt) for d in ldims]
        lay = [od[l].new_layer() for l in range(L)]

        def split(l, img):
            od[l].write_frame_to_chunks(0, img, *lay[l])

    outs = [np.empty((ld[-2][1], ld[-1][1]), dtype=ob.NP_DTYPES[dt]) for ld in ldims]
    n = 0
    t0 = time.perf_counter()
    while True:
        fr = frames[n % len(frames)]
        split(0, fr)
        ds.add_frame(fr)
        for l in range(1, L):
            img = ds.take_frame(l)
            if img is not None:
                split(l, img)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 3:
            break
    if kind == "reference":
        for s in sp:
            R.ref_split_destroy(s)
    gbs = n * frames[0].nbytes / el / 1e9
    if kind == "reference":
        threads = int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))
        how = (f"Downsampler::add_frame+take_frame ({L} levels) on the one consumer "
               f"thread + the tile split of every level with OpenMP over tiles "
               f"(array.cpp:575) on {threads} threads")
    else:
        threads = 1
        how = f"C port: downsample ({L} levels) + tile split of every level, single thread"
    return {"value": round(gbs, 4), "unit": "GB/s", "cores": threads, "kind": kind,
            "downsample_threads": 1, "split_threads": threads,
            "nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "cpu_model": cpu_model(),
            "sample": f"{n} frames of {h}x{w} {ob.DTYPE_NAMES[dt]} ({el:.1f} s): {how}"}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def reduce_dev(dist, dev):
    """Where the max-over-ranks tensor lives: the GPU under RCCL, the CPU
    under gloo."""
    return dev if dist.get_backend() == "nccl" else "cpu"


def run_e2e(torch, aqz, dev, cfg, args, world, rank, dist):
    """Host frame buffer -> H2D -> stage -> D2H of every completed chunk layer
    (the path BASELINE.json asks to be measured end to end).  The source is a
    2-batch ring of host frames; layers land in a per-level ring of pinned
    buffers (no consumer: the sink is out of scope).  Timed from the first
    append to the last hand-off copy."""
    # (the device-resident launch size of C2 is 256 frames; the host path
    # keeps 128-frame batches: a 2-batch pinned source ring of 2 GiB)
    dt, bpp = cfg["dtype"], BPP[cfg["dtype"]]
    B = args.batch or min(cfg["batch"], 128)
    codec = {"none": 0, "lz4": 1, "blosc-zstd": 2, "zstd": 3}[args.codec]
    # a raw hand-off splits level 0 on the host from the frames it holds
    # (H2D 1x, D2H 1/3x of the input instead of 4/3x)
    host0 = args.level0_split == "host" or (args.level0_split == "auto" and not codec)
    if host0 and codec:
        sys.exit("--level0-split host needs a raw hand-off (the codecs compress level 0 "
                 "on the device)")
    st = aqz.Stage(cfg["dims"], dt, cfg["method"], force_levels=cfg["force_levels"],
                   max_batch_frames=B, layer_slots=2, device=dev.index,
                   level0_split_on_host=host0, **args.tune)
    L = st.n_levels()
    sizes = level_sizes(st)
    fbytes = sizes[0][0] * sizes[0][1] * bpp
    lay = [st.layout(l) for l in range(L)]
    lbytes = [x["bytes_per_chunk"] * x["chunks_per_layer"] for x in lay]
    src_frames = 2 * B
    if args.e2e == "pinned":
        src = aqz.HostBuffer(src_frames * fbytes)
        src_arr, src_ptr, mem = src.array, src.ptr, aqz.MEM_HOST_PINNED
    else:
        src_arr = np.empty(src_frames * fbytes, dtype=np.uint8)
        src_ptr, mem = src_arr.ctypes.data, aqz.MEM_HOST
    rng = np.random.default_rng(7 + rank)
    host_zstd = os.environ.get("AQZ_ZSTD_HOST", "0") not in ("", "0")
    if codec:
        # compressible camera-like frames (smooth background + noise)
        n_px = src_arr.size // bpp
        v = 1000.0 + 200.0 * np.sin(np.arange(n_px) / 977.0) + rng.normal(0, 30.0, n_px)
        npdt = {U8: np.uint8, U16: np.uint16, F32: np.float32}[dt]
        if dt == U8:
            v = v / 8.0
        src_arr[...] = v.clip(0, 65535).astype(npdt).view(np.uint8)
    else:
        src_arr[...] = rng.integers(0, 256, size=src_arr.size, dtype=np.uint8)
    cap = [lbytes[l] + 16 * lay[l]["chunks_per_layer"] for l in range(L)]
    dst = [[aqz.HostBuffer(cap[l]) for _ in range(4)] for l in range(L)]
    hd = [[aqz.HostBuffer(lay[l]["chunks_per_layer"]) for _ in range(4)] for l in range(L)]
    handed = [0] * L
    d2h = [0]
    out_bytes = [0]  # bytes handed to the sink (frames or raw chunks)
    pending = []  # compressed layers whose frames are not copied yet

    def drain_compressed():
        while pending:
            l, layer = pending.pop(0)
            i = layer % 4
            off = st.compressed_offsets(l, layer)
            st.copy_compressed_async(l, layer, dst[l][i].ptr, cap[l])
            # PCIe bytes: the frames (device codecs) or the shuffled layer
            # (AQZ_ZSTD_HOST=1: zstd on the host pool)
            d2h[0] += lbytes[l] if codec != 1 and host_zstd else int(off[-1])
            out_bytes[0] += int(off[-1])

    # zstd level 1 (the reference's examples and tests compress at level 1),
    # blosc clevel 5; --clevel overrides
    clevel = args.clevel if args.clevel >= 0 else (1 if codec == 3 else 5)

    appended = [0]

    def split_level0(ptr):
        """Level 0 of the batch at ptr, split on the host into the layer
        buffers (the stage's host threads, next to the device)."""
        F = lay[0]["frames_per_layer"]
        f, end = appended[0], appended[0] + B
        while f < end:
            layer = f // F
            hi = min(end, (layer + 1) * F)
            i = layer % 4
            if f % F == 0:
                hd[0][i].array[...] = 0
            st.split_level0_host(ptr + (f - appended[0]) * fbytes, hi - f, f, dst[0][i].ptr,
                                 lbytes[0], hd[0][i].ptr, hd[0][i].nbytes)
            if hi % F == 0:
                out_bytes[0] += lbytes[0]
                handed[0] += 1
            f = hi
        appended[0] = end

    def hand_off():
        if codec:
            drain_compressed()  # last step's layers: their kernels are done by now
        for l in range(1 if host0 else 0, L):
            done = st.frames_written(l) // lay[l]["frames_per_layer"]
            while handed[l] < done:
                i = handed[l] % 4
                if codec:
                    st.compress_layer(l, handed[l], codec=codec, clevel=clevel,
                                      shuffle=0 if codec == 3 else args.compress)
                    pending.append((l, handed[l]))
                else:
                    st.copy_layer_async(l, handed[l], dst[l][i].ptr, lbytes[l],
                                        hd[l][i].ptr, hd[l][i].nbytes)
                    d2h[0] += lbytes[l]
                    out_bytes[0] += lbytes[l]
                handed[l] += 1

    def step(s):
        ptr = src_ptr + (s % 2) * B * fbytes
        st.append_ptr(ptr, B, mem)
        if host0:
            split_level0(ptr)  # overlaps the batch's H2D and kernels
        hand_off()

    for s in range(args.warmup):
        step(s)
    drain_compressed()
    st.wait_copies()
    st.synchronize()
    if dist:
        dist.barrier()
    d2h[0] = 0
    out_bytes[0] = 0
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(args.warmup + s)
    drain_compressed()
    st.wait_copies()
    st.synchronize()
    el = time.perf_counter() - t0
    if dist:
        dist.barrier()
        t = torch.tensor([el], dtype=torch.float64, device=reduce_dev(dist, dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    affinity = st.host_affinity()
    st.close()
    in_bytes = args.steps * B * fbytes
    return {
        "metric": "end-to-end input GB/s, host frames -> H2D -> multiscale stage -> "
                  + ({1: "device blosc-lz4 compression (shuffle %d) -> D2H of every "
                         "compressed chunk layer" % args.compress,
                      2: ("device shuffle (%d) -> D2H -> host blosc-zstd of every chunk "
                          "layer" if host_zstd else "device blosc-zstd compression "
                          "(shuffle %d) -> D2H of every compressed chunk layer") % args.compress,
                      3: ("D2H -> host zstd of every chunk layer" if host_zstd
                          else "device zstd compression -> D2H of every compressed chunk "
                          "layer")}[codec]
                     if codec else ("level 0 tile-split on the host, D2H of every chunk "
                                    "layer of levels >= 1" if host0
                                    else "D2H of every chunk layer")),
        "value": round(world * in_bytes / el / 1e9, 3), "unit": "GB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el * 1e3 / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": {U8: "u8", U16: "u16", F32: "f32"}[dt],
        "data": f"synthetic{' camera-like' if codec else ' random'}, host {args.e2e} source ring of {src_frames} frames",
        "config": {"workload": cfg["workload"].replace("device-resident", "host-resident") +
                   f" [e2e, {args.e2e} source]", "frames_per_step_per_gpu": B,
                   "levels": L, "clevel": clevel if codec else None},
        "h2d_gbs_per_gpu": round(in_bytes / el / 1e9, 3),
        "d2h_gbs_per_gpu": round(d2h[0] / el / 1e9, 3),
        "frames_per_s_per_gpu": round(args.steps * B / el, 1),
        "host_threads": {"numa_node": affinity[0], "pinned_cpus": affinity[1]},
        "d2h_bytes_per_input_byte": round(d2h[0] / in_bytes, 4),
        "level0_split": "host" if host0 else "device",
        "sink_bytes_per_input_byte": round(out_bytes[0] / in_bytes, 4),
    }


def run_paced(torch, aqz, dev, cfg, args):
    """Simulated camera: frame i lands in a pinned ring of R frames at
    t0 + i/fps (its pixels are the ring's synthetic contents).  The consumer
    appends every batch of b frames as soon as it has landed and hands off
    completed chunk layers; a frame overwritten by the camera before it was
    appended is a drop.  Latency = from the arrival of a batch's last frame
    to the completion of its kernels."""
    dt, bpp = cfg["dtype"], BPP[cfg["dtype"]]
    b = args.batch or 8
    st = aqz.Stage(cfg["dims"], dt, cfg["method"], force_levels=cfg["force_levels"],
                   max_batch_frames=b, layer_slots=3, device=dev.index, **args.tune)
    stream = torch.cuda.Stream(dev)
    st.set_stream(stream.cuda_stream)
    L = st.n_levels()
    sizes = level_sizes(st)
    fbytes = sizes[0][0] * sizes[0][1] * bpp
    lay = [st.layout(l) for l in range(L)]
    lbytes = [x["bytes_per_chunk"] * x["chunks_per_layer"] for x in lay]
    # a quarter second of camera buffer (--camera-ring overrides)
    R = args.camera_ring or max(4 * b, int(args.fps * 0.25))
    ring = aqz.HostBuffer(R * fbytes)
    frame = np.random.default_rng(3).integers(0, 256, size=fbytes, dtype=np.uint8)
    ring.array.reshape(R, fbytes)[:] = frame  # pixel values do not change the cost
    dst = [[aqz.HostBuffer(lbytes[l]) for _ in range(4)] for l in range(L)]
    handed = [0] * L

    def hand_off():
        for l in range(L):
            done = st.frames_written(l) // lay[l]["frames_per_layer"]
            while handed[l] < done:
                st.copy_layer_async(l, handed[l], dst[l][handed[l] % 4].ptr, lbytes[l])
                handed[l] += 1

    n_total = int(args.fps * args.seconds)
    period = 1.0 / args.fps
    consumed, drops, done_frames, appended = 0, 0, 0, 0
    inflight, lat = [], []
    t0 = time.perf_counter() + 0.05
    while consumed < n_total:
        now = time.perf_counter()
        arrived = min(n_total, int((now - t0) / period) + 1) if now >= t0 else 0
        # ring slots held: landed but not appended + appended but not yet
        # read by the stage's DMA; a frame finding no free slot is dropped
        held = (arrived - consumed) + (appended - st.frames_consumed())
        if held > R:
            drops += held - R
            consumed += held - R
        if arrived - consumed >= b or (arrived == n_total and arrived > consumed):
            n = min(b, arrived - consumed)
            s0 = consumed % R
            first = min(n, R - s0)
            st.append_ptr(ring.ptr + s0 * fbytes, first, aqz.MEM_HOST_PINNED)
            if n > first:
                st.append_ptr(ring.ptr, n - first, aqz.MEM_HOST_PINNED)
            ev = torch.cuda.Event()
            ev.record(stream)
            inflight.append((ev, t0 + (consumed + n - 1) * period, n))
            consumed += n
            appended += n
            hand_off()
        else:
            time.sleep(min(period / 4, 0.0005))
        while inflight and inflight[0][0].query():
            ev, t_arr, n = inflight.pop(0)
            lat.append(time.perf_counter() - t_arr)
            done_frames += n
    st.synchronize()
    for ev, t_arr, n in inflight:
        lat.append(time.perf_counter() - t_arr)
        done_frames += n
    el = time.perf_counter() - t0
    frames_written0 = st.frames_written(0)
    st.close()
    lat_ms = np.array(lat) * 1e3
    return {
        "metric": f"sustained fps, simulated camera at {args.fps:g} fps into pinned memory "
                  "-> H2D -> multiscale stage -> D2H of every chunk layer",
        "value": round(done_frames / el, 1), "unit": "frames/s", "n_gpus": 1,
        "higher_is_better": True, "target_fps": args.fps, "frames": n_total,
        "processed": done_frames, "drops": drops, "batch": b, "camera_ring_frames": R,
        "appended": appended, "stage_frames_written": frames_written0,
        "latency_ms": {"p50": round(float(np.percentile(lat_ms, 50)), 2),
                       "p99": round(float(np.percentile(lat_ms, 99)), 2),
                       "max": round(float(lat_ms.max()), 2)},
        "input_gbs": round(done_frames * fbytes / el / 1e9, 3),
        "dtype": {U8: "u8", U16: "u16", F32: "f32"}[dt],
        "config": {"workload": cfg["workload"].replace("device-resident", "host-resident") +
                   f" [paced camera {args.fps:g} fps]", "levels": L},
    }


def self_launch(n):
    """`bench.py --gpus N` without a launcher: run this same command under
    torch.distributed.run with N ranks on 127.0.0.1 (one process per GPU)
    as a child process; rank 0 prints the JSON line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pyramid-only", action="store_true",
                    help="skip the level-0 tile split (downsample levels only)")
    ap.add_argument("--no-pyramid-only-line", action="store_true",
                    help="do not add the pyramid-only side measurement")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="diagnostic: roofline.achieved from the wall time per launch "
                         "instead of the HIP events bracketing the timed region")
    ap.add_argument("--fps", type=float, default=0.0,
                    help="with --e2e pinned: a simulated camera delivering frames "
                         "at this rate into a pinned ring (SURVEY 8d, C3 @ 500 fps); "
                         "reports sustained fps, drops and latency")
    ap.add_argument("--seconds", type=float, default=5.0,
                    help="duration of the --fps run")
    ap.add_argument("--camera-ring", type=int, default=0,
                    help="--fps run: frames in the simulated camera's pinned ring "
                         "(default a quarter second)")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per append (default: the config's batch)")
    ap.add_argument("--compress", type=int, default=0, choices=[0, 1, 2],
                    help="e2e: compress every chunk layer (blosc shuffle: 1 = byte, "
                         "2 = bit) and hand off the frames; implies --codec lz4 "
                         "unless --codec says otherwise")
    ap.add_argument("--codec", default="none",
                    choices=["none", "lz4", "blosc-zstd", "zstd"],
                    help="e2e: chunk codec (lz4: blosc1-lz4 on the device; blosc-zstd "
                         "and zstd: device shuffle + host zstd pool)")
    ap.add_argument("--e2e", choices=["pinned", "pageable"], default=None,
                    help="end-to-end mode: frames start in host memory (pinned or "
                         "pageable), every completed chunk layer is handed back to "
                         "pinned host buffers (DESIGN.md 'End to end')")
    ap.add_argument("--level0-split", choices=["auto", "host", "device"], default="auto",
                    help="e2e: where level 0 is tile-split (auto: on the host for a raw "
                         "hand-off, aqz_stage_options.level0_split_on_host; on the device "
                         "when the layers are compressed there)")
    ap.add_argument("--clevel", type=int, default=-1,
                    help="e2e compression level (default: zstd 1, blosc 5)")
    ap.add_argument("--xy", action="store_true",
                    help="XY-transposed storage order (storage_dimension_order swaps the "
                         "last two dims; the frames stay in acquisition order)")
    ap.add_argument("--no-hbm-probe", action="store_true",
                    help="skip the live streaming probe of this device's HBM rates")
    ap.add_argument("--placement-tries", type=int, default=PLACEMENT["placement_tries"],
                    help="aqz_stage_options.placement_tries of the device-resident stages "
                         "(0: keep the first allocation)")
    ap.add_argument("--tune", action="append", default=[], metavar="FIELD=VALUE",
                    help="bench-header stage option (aqz_stage_bench_options field, e.g. "
                         "knobs=8, nt=3, placement_reps=20); repeatable")
    ap.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    args.tune = {k: int(v, 0) for k, v in (t.split("=", 1) for t in args.tune)}
    if args.codec == "none" and args.compress:
        args.codec = "lz4"

    if args.gpus < 1:
        sys.exit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # No launcher: start one rank per GPU ourselves, before this process
        # has touched the GPU, and exit with the launcher's status.
        sys.exit(self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"--gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU required")
    if args.launch_probe:
        # CPU test hook: report the rank layout -- and for C4 the rank's z
        # slab -- and stop before any GPU work; one write() per line: ranks
        # share the pipe
        probe = {"rank": int(os.environ.get("RANK", "0")), "world": world,
                 "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}
        if args.config == "c4" and world > 1:
            import aqz
            from aqz.dist import z_levels, z_slab
            planes = [lv[1][1] for lv in aqz.pyramid_levels(CONFIGS["c4"]["dims"])]
            probe["z_slab"] = list(z_slab(planes[0], world, probe["rank"],
                                          1 << z_levels(planes)))
        sys.stdout.write(json.dumps(probe) + "\n")
        sys.stdout.flush()
        return

    import torch
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        # nccl (= RCCL) on a real node; AQZ_DIST_BACKEND=gloo rehearses the
        # multi-rank path with ranks sharing the GPUs present
        backend = os.environ.get("AQZ_DIST_BACKEND", "nccl")
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    import aqz
    cfg = CONFIGS[args.config]
    dt = cfg["dtype"]
    B = args.batch or cfg["batch"]
    bpp = BPP[dt]
    slab = None
    planes = None
    if args.config == "c4" and world > 1:
        from aqz.dist import z_levels, z_slab
        planes = [lv[1][1] for lv in aqz.pyramid_levels(cfg["dims"])]
        slab = z_slab(planes[0], world, rank, 1 << z_levels(planes))

    def run(pyramid_only, steps, warmup):
        """Time `steps` launches of B frames (after `warmup`) between
        barrier + device sync on both sides; max over ranks."""
        kw = dict(force_levels=cfg["force_levels"], max_batch_frames=B,
                  layer_slots=layer_slots_for(cfg, B),
                  skip_level0_split=pyramid_only, placement_tries=args.placement_tries)
        kw.update(args.tune)
        if args.xy:
            nd = len(cfg["dims"])
            kw["storage_order"] = list(range(nd - 2)) + [nd - 1, nd - 2]
        est = aqz.estimate_memory(cfg["dims"], dt, cfg["method"], **kw)
        tc = time.perf_counter()
        st = aqz.Stage(cfg["dims"], dt, cfg["method"], device=dev.index, z_slab=slab, **kw)
        # what creation costs a rank: wall time (with the placement search)
        # and the process's peak host RSS so far
        create_s = time.perf_counter() - tc
        rss_mib = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0
        # the stage runs on its own HIP stream; the timing marks below are
        # recorded by the library on that same stream
        sizes = level_sizes(st)
        fbytes = sizes[0][0] * sizes[0][1] * bpp
        ring_frames = cfg["ring"]
        ring = torch.empty(ring_frames * fbytes, dtype=torch.uint8, device=dev)
        fill_ring(torch, ring, dt, 1234 + rank)
        torch.cuda.synchronize(dev)  # torch's stream filled it; the stage's reads it
        nb = ring_frames // B
        base = ring.data_ptr()

        def step(s):
            st.append_ptr(base + (s % nb) * B * fbytes, B)

        for s in range(warmup):
            step(s)
        st.synchronize()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        # one HIP event pair, recorded by the library on the stream the
        # kernels are launched on, brackets the timed region (a pair per
        # launch would add ~10 us of gap per launch to the wall time)
        fw0 = [st.frames_written(l) for l in range(len(sizes))]
        t0 = time.perf_counter()
        st.timing_mark(0)
        for s in range(steps):
            step(warmup + s)
        st.timing_mark(1)
        st.synchronize()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        if dist:
            dist.barrier()
        elapsed = t1 - t0
        elapsed_local = elapsed
        if dist:
            t = torch.tensor([elapsed], dtype=torch.float64, device=reduce_dev(dist, dev))
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        kms, launches = st.timing_elapsed(), steps
        if args.no_kernel_events:
            kms = elapsed * 1e3
        kernel = st.dominant_kernel()
        numa = st.host_affinity()  # (NUMA node of the device, CPUs there)
        placement = st.placement()
        placement["estimate_device_bytes"] = est["device_bytes"]
        placement["stage_create_s"] = round(create_s, 3)
        placement["host_peak_rss_mib"] = round(rss_mib, 1)
        placement["rings_bytes"] = sum(
            x["chunk_pitch"] * x["chunks_per_layer"] * x["layer_slots"]
            for x in (st.layout(l) for l in range(len(sizes))))
        # algorithmic bytes per launch: every input frame read once, plus
        # every frame each level emitted in the timed region written once
        # (a z-halving level emits half as many frames as its parent)
        if slab:  # frame ids jump over other ranks' planes: count planes
            emitted = [steps * B * planes[l] // planes[0] for l in range(len(sizes))]
        else:
            emitted = [st.frames_written(l) - fw0[l] for l in range(len(sizes))]
        st.close()
        del ring
        out_bytes = sum(n * h * w * bpp for n, (h, w) in zip(emitted[1:], sizes[1:]))
        alg = (emitted[0] * fbytes * (1 if pyramid_only else 2) + out_bytes) // max(1, steps)
        avg_ms = kms / max(1, launches)
        return dict(elapsed=elapsed, elapsed_local=elapsed_local, sizes=sizes, fbytes=fbytes,
                    kernel=kernel, numa=numa,
                    avg_ms=avg_ms, alg=alg, placement=placement,
                    achieved=alg / (avg_ms * 1e-3) / 1e9 if launches else 0.0,
                    value=world * steps * B * fbytes / elapsed / 1e9)

    if args.e2e and args.fps > 0:
        res = run_paced(torch, aqz, dev, cfg, args)
        print(json.dumps(res), flush=True)
        return
    if args.e2e:
        res = run_e2e(torch, aqz, dev, cfg, args, world, rank, dist)
        if rank == 0:
            print(json.dumps(res), flush=True)
        if dist:
            dist.destroy_process_group()
        return

    main_run = run(args.pyramid_only, args.steps, args.warmup)
    per_rank = None
    if dist:
        # every rank's own kernel time, placement and creation cost, gathered
        # after the timed region (a few numbers per rank) so a multi-GPU line
        # shows which rank set the max
        mp = main_run["placement"]
        numa = main_run.get("numa")
        mine = {"rank": rank, "device": dev.index, "numa_node": numa[0] if numa else None,
                "host_cpus": numa[1] if numa else None,
                "kernel_avg_ms": round(main_run["avg_ms"], 5),
                "frac": round(main_run["achieved"] / HBM_PEAK_GBS, 4),
                "elapsed_s": round(main_run["elapsed_local"], 5),
                "candidates_ms": mp.get("candidates_ms"), "kept": mp.get("kept"),
                "accepted": mp.get("accepted"), "expected_ms": mp.get("expected_ms"),
                "probe_bus_gbs": mp.get("probe_bus_gbs"),
                "peak_device_bytes": mp.get("peak_device_bytes"),
                "stage_create_s": mp.get("stage_create_s")}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    side = None
    if not args.pyramid_only and not args.no_pyramid_only_line:
        side = run(True, max(5, args.steps // 2), 2)
    probe = None
    if not args.no_hbm_probe:
        probe = hbm_probe(aqz, dev.index)
    sizes, elapsed, value = main_run["sizes"], main_run["elapsed"], main_run["value"]
    kernel, avg_ms, achieved = main_run["kernel"], main_run["avg_ms"], main_run["achieved"]
    alg_per_launch = main_run["alg"]
    pl = main_run["placement"]
    pl["placement_tries"] = args.placement_tries
    # how the chunk-layer rings were allocated (aqz_placement_report.mode)
    pl["ring_allocation"] = ring_allocation(pl)
    traffic, traffic_src, prof = pmc_traffic(args.config, args.pyramid_only, kernel, B,
                                             pl["ring_allocation"], avg_ms, lib_sha256(),
                                             lib_device_code_sha256())

    result = {
        "metric": f"input GB/s, device-resident multiscale downsample, {DTYPE_WORDS[dt]} "
                  "frames @1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {U8: "u8", U16: "u16", F32: "f32"}[dt],
        "data": "synthetic (device-resident random frames, per-rank seed)",
        "config": {"workload": cfg["workload"] + (" [pyramid only: no level-0 split]"
                                                  if args.pyramid_only else "")
                               + (" [XY-transposed storage order]" if args.xy else ""),
                   "frames_per_step_per_gpu": B, "levels": len(sizes),
                   "level_sizes": [f"{h}x{w}" for (h, w) in sizes],
                   "parallelism": f"{world} independent per-GPU streams, no collective"
                                  + (f"; rank r owns z slab [lo, hi) of every "
                                     f"{planes[0]}-plane volume (rank 0: {list(slab)})"
                                     if slab else "")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "traffic_unit": "bytes per launch (rocprofv3 PMC)",
                     "traffic_source": traffic_src,
                     "kernel": kernel,
                     "kernel_avg_ms": round(avg_ms, 5),
                     "alg_bytes_per_launch": alg_per_launch,
                     # creation-time placement search of the chunk-layer rings:
                     # ms per launch of each candidate (random frames), the one
                     # kept, its re-time alone, the creation peak vs estimate
                     "placement": main_run["placement"]},
        "input_rate_frac_of_peak": round(value / world / HBM_PEAK_GBS, 4),
    }
    if prof:
        result["roofline"]["traffic_profile_same_build"] = bool(
            prof.get("lib_sha256") and prof.get("lib_sha256") == lib_sha256())
        result["roofline"]["traffic_profile_same_device_code"] = bool(
            prof.get("device_code_sha256")
            and prof.get("device_code_sha256") == lib_device_code_sha256())
        # the profiled run of this command: its rocprof kernel average and
        # the frac it gives, next to this run's
        pa = prof.get("steady_avg_duration_ns") or prof.get("avg_duration_ns")
        pa *= B / (prof.get("frames_per_launch") or B)
        result["roofline"]["profile_kernel_avg_ms"] = round(pa / 1e6, 5)
        result["roofline"]["profile_frac"] = round(
            alg_per_launch / (pa * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)
    if pl.get("kept_ms_final"):
        # the steady state against the kept placement's own re-time
        pl["steady_over_kept_final"] = round(avg_ms / pl["kept_ms_final"], 4)
    if pl.get("candidates_ms"):
        # candidate 0 is the first allocation: what a stage created without
        # the search (placement_tries 0) runs at -- reported beside the kept
        # one with the same weight (same random frames, same launches)
        c0 = pl["candidates_ms"][0]
        result["roofline"]["candidate0_ms"] = c0
        result["roofline"]["frac_at_candidate0"] = round(
            alg_per_launch / (c0 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        result["roofline"]["kept_ms"] = pl["candidates_ms"][pl["kept"]]
    pg = pl.get("candidates_probe_gbs") or []
    if pl.get("kept", 0) < len(pg) and pg[pl["kept"]] > 0:
        # a reference rate, not a ceiling: the best of three plain streaming
        # kernels of the stage's bus shape (1 read : 4/3 write; nontemporal
        # 96 / 192 B per lane, plain stores) reading the random frames and
        # writing the kept rings, launches of this size, timed at creation
        # (aqz_placement_report.probe_gbs).  The fused kernel runs at about
        # 1.00-1.02 of it: it interleaves its reads and writes over the HBM
        # channels at least as well as a copy loop does.
        result["roofline"]["probe_same_shape_gbs"] = pg[pl["kept"]]
        result["roofline"]["probe_same_shape_source"] = (
            ("read-third" if args.pyramid_only else "copy-third") +
            " streaming kernels over the kept rings' memory at this launch size "
            "(aqz_placement_report.probe_gbs)")
        result["roofline"]["frac_of_probe_same_shape"] = round(achieved / pg[pl["kept"]], 4)
    if probe:
        # this device's streaming rates on separate buffers:
        # 512 MiB launches over a 2 GiB source, so the MALL holds part of
        # their working set -- a characterisation of the box, not a ceiling
        result["hbm_probe"] = probe
    if side:
        # the downsample alone (no level-0 tile split): reads each frame once
        # and writes 1/3 of it; its input rate against the HBM read peak is
        # the "read roofline" fraction of BASELINE.json's target
        result["pyramid_only"] = {
            "value": round(side["value"], 2), "unit": "GB/s",
            "kernel_avg_ms": round(side["avg_ms"], 5),
            "achieved": round(side["achieved"], 1),
            "input_rate_frac_of_peak": round(side["value"] / world / HBM_PEAK_GBS, 4)}
        if probe:
            # a plain streaming kernel of the same shape (1 read : 1/3
            # write) on separate buffers, this run: a reference rate
            pr = probe["read_third_input_gbs"]
            result["pyramid_only"].update({
                "probe_input_gbs": pr,
                "input_rate_frac_of_probe": round(side["value"] / world / pr, 4),
                # kernel time only (no launch gaps): input bytes per launch
                # over the event-timed launch duration
                "kernel_input_frac_of_probe": round(
                    B * side["fbytes"] / (side["avg_ms"] * 1e-3) / 1e9 / pr, 4),
                "probe_source": "hbm_probe.read_third_input_gbs"})
        spl = side["placement"]
        spg = spl.get("candidates_probe_gbs") or []
        if spl.get("kept", 0) < len(spg) and spg[spl["kept"]] > 0:
            # the read-third probe (1 read : 1/3 write) over this stage's own
            # kept rings, from the random frames, at this launch size: the
            # same-memory reference rate of the pyramid-only shape
            result["pyramid_only"].update({
                "probe_same_memory_bus_gbs": spg[spl["kept"]],
                "kernel_frac_of_probe_same_memory": round(
                    side["achieved"] / spg[spl["kept"]], 4),
                "placement_candidates_ms": spl.get("candidates_ms"),
                "placement_kept": spl.get("kept")})
    if per_rank:
        result["per_rank"] = per_rank
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
