"""Python binding of the MI355X multiscale stage (C ABI: include/aqz_gpu.h).

Thin ctypes layer used by tests/ and bench.py.  The compute runs in the HIP
library ``acquire-zarr_amd/libaqz_gpu.so``; there is no CPU fallback -- if the
library is missing and cannot be built, importing this module raises.

Mirrors the reference interfaces:
  Dims         <- ArrayDimensions   (src/streaming/array.dimensions.hh:45)
  Downsampler  <- zarr::Downsampler (src/streaming/downsampler.hh:12-64)
  Stage        <- MultiscaleArray::write_frame hot path
                  (src/streaming/multiscale.array.cpp:57-74, 291-325)
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# AQZ_LIB: dev A/B of two builds in separate processes (tools/); default in-tree
LIB_PATH = os.environ.get("AQZ_LIB") or os.path.join(PKG_DIR, "libaqz_gpu.so")

UINT8, UINT16, UINT32, UINT64, INT8, INT16, INT32, INT64, FLOAT32, FLOAT64 = range(10)
DECIMATE, MEAN, MIN, MAX = range(4)
SPACE, CHANNEL, TIME, OTHER = range(4)
MEM_HOST, MEM_DEVICE, MEM_HOST_PINNED = 0, 1, 2

NP_DTYPES = {UINT8: np.uint8, UINT16: np.uint16, UINT32: np.uint32,
             UINT64: np.uint64, INT8: np.int8, INT16: np.int16,
             INT32: np.int32, INT64: np.int64, FLOAT32: np.float32,
             FLOAT64: np.float64}

STATUS = {0: "Success", 1: "InvalidArgument", 2: "Overflow", 3: "InvalidIndex",
          4: "NotYetImplemented", 5: "InternalError", 6: "OutOfMemory",
          9: "InvalidSettings", 12: "WriteOutOfBounds"}


class AqzError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        super().__init__(f"{what}: {STATUS.get(status, status)} ({status})")
        self.status = status


class Dimension(C.Structure):
    _fields_ = [("type", C.c_int32), ("array_size_px", C.c_uint32),
                ("chunk_size_px", C.c_uint32),
                ("shard_size_chunks", C.c_uint32)]


class ArrayDescC(C.Structure):
    _fields_ = [("dimensions", C.POINTER(Dimension)),
                ("dimension_count", C.c_size_t),
                ("data_type", C.c_int32), ("multiscale", C.c_int32),
                ("downsampling_method", C.c_int32),
                ("max_levels", C.c_uint32),
                ("storage_dimension_order", C.POINTER(C.c_size_t)),
                ("device", C.c_int32)]


class StageOptionsC(C.Structure):
    _fields_ = [("layer_slots", C.c_uint32), ("max_batch_frames", C.c_uint32),
                ("first_frame", C.c_uint64), ("z_slab_begin", C.c_uint32),
                ("z_slab_end", C.c_uint32), ("placement_tries", C.c_uint32),
                ("level0_split_on_host", C.c_uint32)]


class StageBenchOptionsC(C.Structure):
    """aqz_stage_bench_options (include/aqz_gpu_bench.h): not drop-in ABI."""
    _fields_ = [("force_levels", C.c_uint32), ("skip_level0_split", C.c_int32),
                ("placement_tries", C.c_uint32),
                ("placement_reps", C.c_uint32), ("placement_flags", C.c_uint32),
                ("knobs", C.c_uint32),
                ("nt_policy", C.c_uint32), ("xcd_rot", C.c_uint32),
                ("region_rows_log2", C.c_uint32), ("zstd_flags", C.c_uint32),
                ("ring_malloc_flags", C.c_uint32), ("chunk_pad_bytes", C.c_uint64),
                ("ring_spacer_bytes", C.c_uint64),
                ("ring_arena_bytes", C.c_uint64)]


# zstd_flags bits of aqz_stage_bench_options
ZSTD_LITERALS_ONLY, ZSTD_NO_FAR, ZSTD_NO_FIT = 1, 2, 4
ZSTD_FAR_ONE_RANGE = 1 << 21  # A/B: no parallel far ranges
BENCH_FIELDS = tuple(f for f, _ in StageBenchOptionsC._fields_ if f != "reserved")


def _bench_options(bench):
    """StageBenchOptionsC from a dict of bench-header fields (None if empty).
    skip_level0_split may be a bool; nt (a policy 0-7) maps to nt_policy."""
    bench = {k: v for k, v in (bench or {}).items() if v}
    if "nt" in bench:
        bench["nt_policy"] = 8 | (bench.pop("nt") & 7)
    if not bench:
        return None
    unknown = set(bench) - set(BENCH_FIELDS)
    if unknown:
        raise TypeError(f"unknown bench options {sorted(unknown)}")
    b = StageBenchOptionsC()
    for k, v in bench.items():
        setattr(b, k, int(v))
    return b


class PlacementReportC(C.Structure):
    """aqz_placement_report (include/aqz_gpu_bench.h)."""
    _fields_ = [("n", C.c_uint32), ("kept", C.c_uint32), ("reps", C.c_uint32),
                ("mode", C.c_uint32), ("ms", C.c_double * 32),
                ("kept_ms_final", C.c_double), ("peak_device_bytes", C.c_uint64),
                ("probe_bus_gbs", C.c_double), ("expected_ms", C.c_double),
                ("alg_bytes", C.c_uint64), ("accepted", C.c_uint32),
                ("stop", C.c_uint32), ("probe_gbs", C.c_double * 32)]


class MemoryUsageC(C.Structure):
    _fields_ = [("device_bytes", C.c_uint64), ("pinned_bytes", C.c_uint64)]


class CompressionC(C.Structure):
    _fields_ = [("codec", C.c_int32), ("clevel", C.c_int32), ("shuffle", C.c_int32)]


CODEC_NONE, CODEC_BLOSC_LZ4, CODEC_BLOSC_ZSTD, CODEC_ZSTD = 0, 1, 2, 3


class ChunkEntryC(C.Structure):
    _fields_ = [("chunk", C.c_uint32), ("shard", C.c_uint32), ("internal", C.c_uint32),
                ("reserved", C.c_uint32), ("offset", C.c_uint64), ("nbytes", C.c_uint64)]


SHARD_UNWRITTEN = (1 << 64) - 1


class LevelLayoutC(C.Structure):
    _fields_ = [("bytes_per_chunk", C.c_uint64),
                ("chunks_per_layer", C.c_uint32), ("layer_slots", C.c_uint32),
                ("frames_per_layer", C.c_uint64), ("frame_bytes", C.c_uint64),
                ("width", C.c_uint32), ("height", C.c_uint32),
                ("chunk_pitch", C.c_uint64)]


def build_library(force: bool = False) -> str:
    """Compile libaqz_gpu.so for gfx950 in-tree (hipcc, no GPU needed)."""
    if force or not os.path.exists(LIB_PATH):
        jobs = str(min(8, os.cpu_count() or 1))
        subprocess.run(["make", "-C", PKG_DIR, "-j" + jobs], check=True,
                       stdout=subprocess.DEVNULL)
    return LIB_PATH


_lib = None


def _preload_hip_runtime():
    """One HIP runtime per process.  PyTorch ships its own libamdhip64
    (soname libamdhip64.so.7) and finds it by path; if this library bound
    /opt/rocm's copy first, a later torch CUDA init would start a second
    runtime and fail.  Loading torch's copy first makes our NEEDED
    libamdhip64.so.7 resolve to it, and torch later re-uses it (same file)."""
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
        if spec is None or not spec.submodule_search_locations:
            return
        p = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
        if os.path.exists(p):
            C.CDLL(p, mode=C.RTLD_GLOBAL)
    except OSError:
        pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    build_library()
    _preload_hip_runtime()
    L = C.CDLL(LIB_PATH)
    vp, sz, i32, u32, u64 = C.c_void_p, C.c_size_t, C.c_int32, C.c_uint32, C.c_uint64
    D = C.POINTER(Dimension)
    sig = {
        "aqz_version": ([], C.c_char_p),
        "aqz_status_message": ([i32], C.c_char_p),
        "aqz_last_error": ([], C.c_char_p),
        "aqz_device_count": ([C.POINTER(i32)], i32),
        "aqz_dims_create": ([D, sz, i32, C.POINTER(sz), C.POINTER(vp)], i32),
        "aqz_dims_destroy": ([vp], None),
        "aqz_dims_ndims": ([vp], sz),
        "aqz_dims_get": ([vp, sz, D], i32),
        "aqz_dims_tile_group_offset": ([vp, u64], u32),
        "aqz_dims_chunk_internal_offset": ([vp, u64], u64),
        "aqz_dims_chunk_lattice_index": ([vp, u64, u32], u32),
        "aqz_dims_transpose_frame_id": ([vp, u64], u64),
        "aqz_dims_bytes_per_chunk": ([vp], u64),
        "aqz_dims_number_of_chunks_in_memory": ([vp], u32),
        "aqz_dims_frames_per_chunk_layer": ([vp], u64),
        "aqz_dims_shard_index_for_chunk": ([vp, u32], u32),
        "aqz_dims_shard_internal_index": ([vp, u32], u32),
        "aqz_dims_shard_geometry": ([vp, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)], i32),
        "aqz_dims_skipped_internal_indices": ([vp, u32, u32, C.POINTER(u32), sz,
                                               C.POINTER(sz)], i32),
        "aqz_pyramid_levels": ([D, sz, u32, C.POINTER(u32), D, sz], i32),
        "aqz_dims_split_frame_rows": ([vp, vp, u64, u32, u32, u32, vp, sz, vp, sz], i32),
        "aqz_stage_split_level0_host": ([vp, vp, u64, u64, u32, vp, sz, vp, sz], i32),
        "aqz_stage_split_level0_rows": ([vp, vp, u64, u32, u32, vp, u32, vp, sz, vp, sz], i32),
        "aqz_dims_dim1_banding": ([vp, C.POINTER(i32), C.POINTER(u32), C.POINTER(u64),
                                   C.POINTER(u32)], i32),
        "aqz_downsampling_method_name": ([i32], C.c_char_p),
        "aqz_downsampling_metadata_json": ([i32, C.c_char_p, sz, C.POINTER(sz)], i32),
        "aqz_downsampler_create": ([C.POINTER(ArrayDescC), C.POINTER(vp)], i32),
        "aqz_downsampler_destroy": ([vp], None),
        "aqz_downsampler_n_levels": ([vp], u32),
        "aqz_downsampler_level_dims": ([vp, u32, D, sz, C.POINTER(sz)], i32),
        "aqz_downsampler_add_frame": ([vp, vp, sz, i32], i32),
        "aqz_downsampler_take_frame": ([vp, u32, vp, sz, i32, C.POINTER(sz), C.POINTER(i32)], i32),
        "aqz_downsampler_method_name": ([vp], C.c_char_p),
        "aqz_downsampler_metadata_json": ([vp, C.c_char_p, sz, C.POINTER(sz)], i32),
        "aqz_stage_create": ([C.POINTER(ArrayDescC), C.POINTER(StageOptionsC), C.POINTER(vp)], i32),
        "aqz_stage_create_bench": ([C.POINTER(ArrayDescC), C.POINTER(StageOptionsC),
                                    C.POINTER(StageBenchOptionsC), C.POINTER(vp)], i32),
        "aqz_stage_wait_stream": ([vp, vp], i32),
        "aqz_stage_band_geometry": ([vp, u32, C.POINTER(i32), C.POINTER(u32), C.POINTER(u64),
                                     C.POINTER(u32)], i32),
        "aqz_stage_copy_band_async": ([vp, u32, u64, u32, vp, sz, vp, sz], i32),
        "aqz_stage_memory_usage": ([vp, C.POINTER(MemoryUsageC)], i32),
        "aqz_stage_estimate_memory": ([C.POINTER(ArrayDescC), C.POINTER(StageOptionsC),
                                       C.POINTER(MemoryUsageC)], i32),
        "aqz_stage_estimate_memory_bench": ([C.POINTER(ArrayDescC), C.POINTER(StageOptionsC),
                                             C.POINTER(StageBenchOptionsC),
                                             C.POINTER(MemoryUsageC)], i32),
        "aqz_stage_placement_report": ([vp, C.POINTER(PlacementReportC)], i32),
        "aqz_stage_destroy": ([vp], None),
        "aqz_stage_n_levels": ([vp], u32),
        "aqz_stage_level_dims": ([vp, u32, D, sz, C.POINTER(sz)], i32),
        "aqz_stage_level_layout": ([vp, u32, C.POINTER(LevelLayoutC)], i32),
        "aqz_stage_set_stream": ([vp, vp], i32),
        "aqz_stage_set_tuning": ([vp, u32, u32], i32),
        "aqz_stage_append": ([vp, vp, u64, i32], i32),
        "aqz_stage_synchronize": ([vp], i32),
        "aqz_stage_frames_written": ([vp, u32], u64),
        "aqz_stage_copy_layer": ([vp, u32, u64, vp, sz, vp, sz, i32], i32),
        "aqz_stage_copy_layer_async": ([vp, u32, u64, vp, sz, vp, sz], i32),
        "aqz_stage_frames_consumed": ([vp], u64),
        "aqz_stage_wait_consumed": ([vp, u64], i32),
        "aqz_stage_last_ticket": ([vp], u64),
        "aqz_stage_copies_completed": ([vp], u64),
        "aqz_stage_wait_ticket": ([vp, u64], i32),
        "aqz_stage_wait_copies": ([vp], i32),
        "aqz_host_alloc": ([sz, C.POINTER(vp)], i32),
        "aqz_host_free": ([vp], None),
        "aqz_stage_device_layer": ([vp, u32, u64, C.POINTER(vp), C.POINTER(vp)], i32),
        "aqz_stage_finalize": ([vp], i32),
        "aqz_stage_enable_kernel_timing": ([vp, i32], i32),
        "aqz_stage_kernel_timing": ([vp, C.POINTER(C.c_double), C.POINTER(u64)], i32),
        "aqz_stage_timing_mark": ([vp, i32], i32),
        "aqz_stage_timing_elapsed": ([vp, C.POINTER(C.c_double)], i32),
        "aqz_stage_dominant_kernel": ([vp], C.c_char_p),
        "aqz_stage_zstd_far_ranges": ([vp, u32], u32),
        "aqz_probe_hbm": ([i32, i32, u64, u32, C.POINTER(C.c_double), C.POINTER(u64)], i32),
        "aqz_stage_placement": ([vp, C.POINTER(C.c_double), sz, C.POINTER(sz),
                                 C.POINTER(u32)], i32),
        "aqz_stage_host_affinity": ([vp, C.POINTER(i32), C.POINTER(u32)], i32),
        "aqz_stage_compress_layer": ([vp, u32, u64, C.POINTER(CompressionC)], i32),
        "aqz_stage_compressed_offsets": ([vp, u32, u64, C.POINTER(u64), sz], i32),
        "aqz_stage_copy_compressed_async": ([vp, u32, u64, vp, sz], i32),
        "aqz_compressor_create": ([u64, u32, C.POINTER(CompressionC), C.POINTER(vp)], i32),
        "aqz_compressor_destroy": ([vp], None),
        "aqz_compressor_max_bytes": ([u64, u32], u64),
        "aqz_compressor_scratch_bytes": ([C.POINTER(CompressionC), u64, u32, u32], u64),
        "aqz_compressor_run": ([vp, vp, u64, u32, vp, sz, vp, vp], i32),
        "aqz_compressor_blocksize": ([vp], u32),
        "aqz_stage_bench_replace_rings": ([vp, u32], i32),
        "aqz_stage_bench_set_ring_offset": ([vp, u64], i32),
        "aqz_stage_bind_host_thread": ([vp], i32),
        "aqz_stage_import_frames": ([vp, vp, u32, u64, u32, u32], i32),
        "aqz_stage_compression_done": ([vp, u32, u64, C.POINTER(C.c_int32)], i32),
        "aqz_stage_compressed_entries": ([vp, u32, u64, C.POINTER(ChunkEntryC), sz], i32),
        "aqz_stage_shard_geometry": ([vp, u32, C.POINTER(u32), C.POINTER(u32),
                                      C.POINTER(u32)], i32),
        "aqz_shard_table_bytes": ([u32], sz),
        "aqz_shard_table": ([vp, vp, u32, vp, sz], i32),
        "aqz_crc32c": ([vp, sz], u32),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _check(status: int, what: str) -> None:
    if status != 0:
        msg = lib().aqz_last_error()
        raise AqzError(status, what + (": " + msg.decode() if msg else ""))


PROBE_READ, PROBE_COPY, PROBE_COPY_THIRD, PROBE_READ_THIRD = 0, 1, 2, 3
PROBE_PLAIN_STORES = 0x100
PROBE_PIECES = 0x200
PROBE_DEEP = 0x400


def probe_hbm(shape: int, nbytes: int = 512 << 20, reps: int = 20, device: int = 0):
    """(ms per launch, bytes read per launch) of the streaming probe
    (aqz_probe_hbm, include/aqz_gpu_bench.h): this device's practical HBM
    rate for one of the stage's access shapes."""
    ms, rd = C.c_double(0), C.c_uint64(0)
    _check(lib().aqz_probe_hbm(device, shape, nbytes, reps, C.byref(ms), C.byref(rd)),
           "aqz_probe_hbm")
    return ms.value, rd.value


def device_count() -> int:
    n = C.c_int32(0)
    _check(lib().aqz_device_count(C.byref(n)), "aqz_device_count")
    return n.value


def _dims_c(dims):
    arr = (Dimension * len(dims))()
    for i, d in enumerate(dims):
        arr[i] = Dimension(*d)
    return arr


def _tuples(arr, n):
    return [(arr[i].type, arr[i].array_size_px, arr[i].chunk_size_px,
             arr[i].shard_size_chunks) for i in range(n)]


class Dims:
    """ArrayDimensions on the host restatement in libaqz_gpu (no GPU)."""

    def __init__(self, dims, dtype, storage_order=None):
        self._keep = _dims_c(dims)
        order = None
        if storage_order is not None:
            order = (C.c_size_t * len(storage_order))(*storage_order)
        h = C.c_void_p()
        _check(lib().aqz_dims_create(self._keep, len(dims), dtype, order,
                                     C.byref(h)), "aqz_dims_create")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.aqz_dims_destroy(self.h)
            self.h = None

    def ndims(self):
        return lib().aqz_dims_ndims(self.h)

    def dims(self):
        out = []
        for i in range(self.ndims()):
            d = Dimension()
            _check(lib().aqz_dims_get(self.h, i, C.byref(d)), "aqz_dims_get")
            out.append((d.type, d.array_size_px, d.chunk_size_px, d.shard_size_chunks))
        return out

    def tile_group_offset(self, fid):
        return lib().aqz_dims_tile_group_offset(self.h, fid)

    def chunk_internal_offset(self, fid):
        return lib().aqz_dims_chunk_internal_offset(self.h, fid)

    def chunk_lattice_index(self, fid, dim):
        return lib().aqz_dims_chunk_lattice_index(self.h, fid, dim)

    def transpose_frame_id(self, fid):
        return lib().aqz_dims_transpose_frame_id(self.h, fid)

    def bytes_per_chunk(self):
        return lib().aqz_dims_bytes_per_chunk(self.h)

    def number_of_chunks_in_memory(self):
        return lib().aqz_dims_number_of_chunks_in_memory(self.h)

    def frames_per_chunk_layer(self):
        return lib().aqz_dims_frames_per_chunk_layer(self.h)

    def shard_index_for_chunk(self, c):
        return lib().aqz_dims_shard_index_for_chunk(self.h, c)

    def shard_internal_index(self, c):
        return lib().aqz_dims_shard_internal_index(self.h, c)

    def shard_geometry(self):
        """(chunks_per_shard, number_of_shards, chunk_layers_per_shard)"""
        a, b, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
        _check(lib().aqz_dims_shard_geometry(self.h, C.byref(a), C.byref(b), C.byref(c)),
               "aqz_dims_shard_geometry")
        return a.value, b.value, c.value

    def skipped_internal_indices(self, shard, layer):
        """ArrayDimensions::skipped_internal_indices_for_shard_layer"""
        n = C.c_size_t(0)
        _check(lib().aqz_dims_skipped_internal_indices(self.h, shard, layer, None, 0,
                                                       C.byref(n)), "skipped_internal")
        out = (C.c_uint32 * max(1, n.value))()
        _check(lib().aqz_dims_skipped_internal_indices(self.h, shard, layer, out, n.value,
                                                       C.byref(n)), "skipped_internal")
        return list(out[:n.value])

    def split_frame_rows(self, frame, frame_id, dst, has_data, row_begin=0, row_end=None,
                         chunk0=0):
        """aqz_dims_split_frame_rows: rows [row_begin, row_end) of one frame
        (numpy, acquisition order) into the packed chunks [chunk0, ...) of a
        layer (numpy uint8 dst, has_data)."""
        frame = np.ascontiguousarray(frame)
        if row_end is None:
            row_end = frame.shape[-2] if frame.ndim >= 2 else 0
        assert dst.dtype == np.uint8 and has_data.dtype == np.uint8
        _check(lib().aqz_dims_split_frame_rows(self.h, frame.ctypes.data, frame_id, row_begin,
                                               row_end, chunk0, dst.ctypes.data, dst.nbytes,
                                               has_data.ctypes.data, has_data.size),
               "aqz_dims_split_frame_rows")

    def dim1_banding(self):
        """(supported, n_bands, frames_per_band, chunks_per_band)"""
        a, b, c, d = C.c_int32(), C.c_uint32(), C.c_uint64(), C.c_uint32()
        _check(lib().aqz_dims_dim1_banding(self.h, C.byref(a), C.byref(b), C.byref(c),
                                           C.byref(d)), "aqz_dims_dim1_banding")
        return bool(a.value), b.value, c.value, d.value


def downsampling_method_name(method):
    """Downsampler::downsampling_method for a method value (no GPU)."""
    return lib().aqz_downsampling_method_name(method).decode()


def downsampling_metadata_json(method):
    """Downsampler::get_metadata().dump() for a method value (no GPU)."""
    n = C.c_size_t(0)
    _check(lib().aqz_downsampling_metadata_json(method, None, 0, C.byref(n)), "metadata")
    buf = C.create_string_buffer(n.value + 1)
    _check(lib().aqz_downsampling_metadata_json(method, buf, n.value + 1, C.byref(n)),
           "metadata")
    return buf.value.decode()


def estimate_memory(dims, dtype, method, max_levels=0, layer_slots=0,
                    max_batch_frames=0, storage_order=None, placement_tries=0,
                    level0_split_on_host=False, **bench):
    """aqz_stage_estimate_memory: upper bound of a stage's footprint (no GPU),
    including the placement search's creation peak when placement_tries > 1.
    With bench-header options (force_levels, skip_level0_split,
    placement_reps, ...), aqz_stage_estimate_memory_bench."""
    d, keep = _desc(dims, dtype, method, max_levels, True, storage_order, 0)
    o = StageOptionsC(layer_slots, max_batch_frames, 0, 0, 0, placement_tries,
                      int(bool(level0_split_on_host)))
    m = MemoryUsageC()
    b = _bench_options(bench)
    if b is not None:
        _check(lib().aqz_stage_estimate_memory_bench(C.byref(d), C.byref(o), C.byref(b),
                                                     C.byref(m)),
               "aqz_stage_estimate_memory_bench")
    else:
        _check(lib().aqz_stage_estimate_memory(C.byref(d), C.byref(o), C.byref(m)),
               "aqz_stage_estimate_memory")
    return {"device_bytes": m.device_bytes, "pinned_bytes": m.pinned_bytes}


def compressor_max_bytes(chunk_bytes, n_chunks):
    """aqz_compressor_max_bytes: bytes that always hold the frames of
    n_chunks chunks of chunk_bytes (any codec; no GPU)."""
    return lib().aqz_compressor_max_bytes(chunk_bytes, n_chunks)


def compressor_scratch_bytes(codec, chunk_bytes, typesize, n_chunks):
    """aqz_compressor_scratch_bytes for codec = (codec, clevel, shuffle)."""
    c = CompressionC(*codec)
    return lib().aqz_compressor_scratch_bytes(C.byref(c), chunk_bytes, typesize, n_chunks)


def pyramid_levels(dims, max_levels=0):
    """Level dims per Downsampler::make_writer_configurations_ (no GPU)."""
    d = _dims_c(dims)
    n = C.c_uint32(0)
    _check(lib().aqz_pyramid_levels(d, len(dims), max_levels, C.byref(n), None, 0),
           "aqz_pyramid_levels")
    nd = max(3, len(dims))
    out = (Dimension * (n.value * nd))()
    _check(lib().aqz_pyramid_levels(d, len(dims), max_levels, C.byref(n), out,
                                    n.value * nd), "aqz_pyramid_levels")
    return [_tuples(out[l * nd:(l + 1) * nd], nd) for l in range(n.value)]


def _desc(dims, dtype, method, max_levels, multiscale, storage_order, device):
    keep = [_dims_c(dims)]
    order = None
    if storage_order is not None:
        order = (C.c_size_t * len(storage_order))(*storage_order)
        keep.append(order)
    d = ArrayDescC(keep[0], len(dims), dtype, 1 if multiscale else 0, method,
                   max_levels, order, device)
    return d, keep


class HostBuffer:
    """Page-locked host memory (aqz_host_alloc) with a numpy view; frames in
    it are appended with MEM_HOST_PINNED (no staging copy) and hand-off
    copies into it overlap the kernels."""

    def __init__(self, nbytes):
        p = C.c_void_p()
        _check(lib().aqz_host_alloc(nbytes, C.byref(p)), "aqz_host_alloc")
        self.ptr = p.value
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(self.ptr))

    def view(self, dtype=np.uint8, shape=None):
        a = self.array.view(dtype)
        return a.reshape(shape) if shape is not None else a

    def close(self):
        if getattr(self, "ptr", None) and _lib is not None:
            self.array = None
            _lib.aqz_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.close()


def _ptr(buf):
    """(pointer, mem kind) for numpy arrays / torch tensors / raw ints."""
    if isinstance(buf, HostBuffer):
        return buf.ptr, MEM_HOST_PINNED
    if isinstance(buf, np.ndarray):
        assert buf.flags.c_contiguous
        return buf.ctypes.data, MEM_HOST
    if hasattr(buf, "data_ptr"):
        assert buf.is_contiguous()
        return buf.data_ptr(), (MEM_DEVICE if buf.is_cuda else MEM_HOST)
    raise TypeError(type(buf))


class Downsampler:
    """zarr::Downsampler on the GPU: add_frame / take_frame."""

    def __init__(self, dims, dtype, method, max_levels=0, storage_order=None,
                 device=0):
        self.dtype = dtype
        d, self._keep = _desc(dims, dtype, method, max_levels, True,
                              storage_order, device)
        h = C.c_void_p()
        _check(lib().aqz_downsampler_create(C.byref(d), C.byref(h)),
               "aqz_downsampler_create")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.aqz_downsampler_destroy(self.h)
            self.h = None

    def n_levels(self):
        return lib().aqz_downsampler_n_levels(self.h)

    def level_dims(self, level):
        out = (Dimension * 16)()
        n = C.c_size_t(0)
        _check(lib().aqz_downsampler_level_dims(self.h, level, out, 16, C.byref(n)),
               "level_dims")
        return _tuples(out, n.value)

    def add_frame(self, frame):
        p, mem = _ptr(frame)
        nbytes = frame.nbytes if isinstance(frame, np.ndarray) else \
            frame.numel() * frame.element_size()
        _check(lib().aqz_downsampler_add_frame(self.h, p, nbytes, mem), "add_frame")

    def take_frame(self, level):
        d = self.level_dims(level) if level < self.n_levels() else None
        if d is None:
            return None
        out = np.empty((d[-2][1], d[-1][1]), dtype=NP_DTYPES[self.dtype])
        nb = C.c_size_t(0)
        found = C.c_int32(0)
        _check(lib().aqz_downsampler_take_frame(self.h, level, out.ctypes.data,
                                                out.nbytes, MEM_HOST,
                                                C.byref(nb), C.byref(found)),
               "take_frame")
        return out if found.value else None

    def method_name(self):
        return lib().aqz_downsampler_method_name(self.h).decode()

    def metadata_json(self):
        n = C.c_size_t(0)
        _check(lib().aqz_downsampler_metadata_json(self.h, None, 0, C.byref(n)), "meta")
        buf = C.create_string_buffer(n.value + 1)
        _check(lib().aqz_downsampler_metadata_json(self.h, buf, n.value + 1, C.byref(n)),
               "meta")
        return buf.value.decode()


class Stage:
    """Device-resident multiscale stage: tile split + pyramid of every level.

    Keyword arguments beyond the drop-in options of include/aqz_gpu.h
    (force_levels, skip_level0_split, knobs, nt, chunk_pad_bytes,
    zstd_flags, placement_reps, ...) are the bench-only fields of
    include/aqz_gpu_bench.h (aqz_stage_create_bench)."""

    def __init__(self, dims, dtype, method, max_levels=0, multiscale=True,
                 storage_order=None, device=0, layer_slots=0,
                 max_batch_frames=0, first_frame=0, z_slab=None,
                 placement_tries=0, level0_split_on_host=False, **bench):
        self.dtype = dtype
        d, self._keep = _desc(dims, dtype, method, max_levels, multiscale,
                              storage_order, device)
        zb, ze = z_slab if z_slab else (0, 0)
        o = StageOptionsC(layer_slots, max_batch_frames, first_frame, zb, ze,
                          placement_tries, int(bool(level0_split_on_host)))
        h = C.c_void_p()
        b = _bench_options(bench)
        if b is not None:
            rc = lib().aqz_stage_create_bench(C.byref(d), C.byref(o), C.byref(b), C.byref(h))
        else:
            rc = lib().aqz_stage_create(C.byref(d), C.byref(o), C.byref(h))
        _check(rc, "aqz_stage_create")
        self.h = h
        self._held = []  # (appended count, CUDA tensor) still being read
        self._appended = 0

    def close(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.aqz_stage_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def n_levels(self):
        return lib().aqz_stage_n_levels(self.h)

    def level_dims(self, level):
        out = (Dimension * 16)()
        n = C.c_size_t(0)
        _check(lib().aqz_stage_level_dims(self.h, level, out, 16, C.byref(n)),
               "level_dims")
        return _tuples(out, n.value)

    def layout(self, level):
        l = LevelLayoutC()
        _check(lib().aqz_stage_level_layout(self.h, level, C.byref(l)), "layout")
        return {f: getattr(l, f) for f, _ in LevelLayoutC._fields_}

    def set_stream(self, stream_ptr):
        _check(lib().aqz_stage_set_stream(self.h, stream_ptr), "set_stream")

    def import_frames(self, src, level, layer, first, count):
        """z-slab assembly: frames [first, first + count) of a chunk layer
        copied from stage `src` (None: zero-filled), aqz_stage_import_frames."""
        _check(lib().aqz_stage_import_frames(self.h, src.h if src is not None else None,
                                             level, layer, first, count), "import_frames")

    def replace_rings(self, level_mask):
        """Bench: fresh chunk-layer rings for the levels in level_mask (the
        old ones stay allocated); placement experiments only."""
        _check(lib().aqz_stage_bench_replace_rings(self.h, level_mask), "replace_rings")

    def set_ring_offset(self, offset):
        """Bench (ring_arena_bytes stages): every ring moved to arena +
        offset; the stage restarts at frame 0."""
        _check(lib().aqz_stage_bench_set_ring_offset(self.h, offset), "set_ring_offset")

    def set_tuning(self, knobs=0, nt=0):
        _check(lib().aqz_stage_set_tuning(self.h, knobs, nt), "set_tuning")

    def append(self, frames, n_frames=None):
        """Append frames from a numpy array (pageable), a HostBuffer (pinned)
        or a torch tensor.  A CUDA tensor is read on the stage's own stream:
        that stream first waits for the work torch has queued on the
        tensor's current stream (no host sync), and the tensor is kept
        alive until the stage reports its frames consumed."""
        p, mem = _ptr(frames)
        if n_frames is None:
            n_frames = frames.shape[0] if frames.ndim == 3 else 1
        cuda = mem == MEM_DEVICE and hasattr(frames, "data_ptr")
        if cuda:
            import torch
            s = torch.cuda.current_stream(frames.device).cuda_stream
            _check(lib().aqz_stage_wait_stream(self.h, s), "wait_stream")
        _check(lib().aqz_stage_append(self.h, p, n_frames, mem), "append")
        self._appended += n_frames
        if cuda:
            self._held.append((self._appended, frames))
        self._release_consumed()

    def append_ptr(self, ptr, n_frames, mem=MEM_DEVICE):
        """Append from a raw pointer; the caller orders and keeps its
        memory (see frames_consumed)."""
        _check(lib().aqz_stage_append(self.h, ptr, n_frames, mem), "append")
        self._appended += n_frames

    def wait_stream(self, stream_ptr):
        _check(lib().aqz_stage_wait_stream(self.h, stream_ptr), "wait_stream")

    def _release_consumed(self):
        if self._held:
            done = self.frames_consumed()
            self._held = [(n, t) for n, t in self._held if n > done]

    def band_geometry(self, level):
        """(supported, n_bands, frames_per_band, chunks_per_band) of dim-1
        banding (Array::flush_completed_bands_)."""
        a, b, c, d = C.c_int32(), C.c_uint32(), C.c_uint64(), C.c_uint32()
        _check(lib().aqz_stage_band_geometry(self.h, level, C.byref(a), C.byref(b),
                                             C.byref(c), C.byref(d)), "band_geometry")
        return bool(a.value), b.value, c.value, d.value

    def copy_band_async(self, level, layer, band, dst_ptr, cap, has_data_ptr=None,
                        has_data_cap=0):
        _check(lib().aqz_stage_copy_band_async(self.h, level, layer, band, dst_ptr, cap,
                                               has_data_ptr, has_data_cap),
               "copy_band_async")

    def memory_usage(self):
        m = MemoryUsageC()
        _check(lib().aqz_stage_memory_usage(self.h, C.byref(m)), "memory_usage")
        return {"device_bytes": m.device_bytes, "pinned_bytes": m.pinned_bytes}

    def synchronize(self):
        _check(lib().aqz_stage_synchronize(self.h), "synchronize")
        self._release_consumed()

    def frames_written(self, level):
        return lib().aqz_stage_frames_written(self.h, level)

    def split_level0_host(self, frames_ptr, n_frames, first_frame, dst_ptr, cap, has_ptr,
                          has_cap, chunk0=0):
        """aqz_stage_split_level0_host: level-0 frames [first_frame, +n) (host
        memory at frames_ptr) tile-split by the stage's host threads into the
        packed chunks [chunk0, ...) of one layer at dst_ptr (host)."""
        _check(lib().aqz_stage_split_level0_host(self.h, frames_ptr, n_frames, first_frame,
                                                 chunk0, dst_ptr, cap, has_ptr, has_cap),
               "split_level0_host")

    def split_level0_rows(self, frame_ptr, frame_id, row_begin, row_end, dst_ptr, cap,
                          has_ptr, has_cap, chunk0=0, frame_copy_ptr=None):
        """aqz_stage_split_level0_rows: rows of one level-0 frame, this thread
        (and, with frame_copy_ptr, the same rows copied there)."""
        _check(lib().aqz_stage_split_level0_rows(self.h, frame_ptr, frame_id, row_begin,
                                                 row_end, frame_copy_ptr, chunk0, dst_ptr, cap,
                                                 has_ptr, has_cap), "split_level0_rows")

    def frames_consumed(self):
        """Level-0 frames whose source bytes have been read (reusable)."""
        return lib().aqz_stage_frames_consumed(self.h)

    def copy_layer(self, level, layer):
        lay = self.layout(level)
        nbytes = lay["bytes_per_chunk"] * lay["chunks_per_layer"]
        out = np.empty(nbytes, dtype=np.uint8)
        flags = np.empty(lay["chunks_per_layer"], dtype=np.uint8)
        _check(lib().aqz_stage_copy_layer(self.h, level, layer, out.ctypes.data,
                                          nbytes, flags.ctypes.data, flags.size,
                                          MEM_HOST), "copy_layer")
        return out, flags

    def copy_layer_async(self, level, layer, dst_ptr, cap, has_data_ptr=None,
                         has_data_cap=0):
        """Enqueue the D2H hand-off of a resident layer (returns at once)."""
        _check(lib().aqz_stage_copy_layer_async(self.h, level, layer, dst_ptr, cap,
                                                has_data_ptr, has_data_cap),
               "copy_layer_async")

    def wait_consumed(self, frames):
        _check(lib().aqz_stage_wait_consumed(self.h, frames), "wait_consumed")
        self._release_consumed()

    def last_ticket(self):
        return lib().aqz_stage_last_ticket(self.h)

    def copies_completed(self):
        return lib().aqz_stage_copies_completed(self.h)

    def wait_ticket(self, ticket):
        _check(lib().aqz_stage_wait_ticket(self.h, ticket), "wait_ticket")

    def wait_copies(self):
        _check(lib().aqz_stage_wait_copies(self.h), "wait_copies")

    def finalize(self):
        _check(lib().aqz_stage_finalize(self.h), "finalize")
        self._release_consumed()

    def enable_kernel_timing(self, on=True):
        _check(lib().aqz_stage_enable_kernel_timing(self.h, 1 if on else 0), "timing")

    def kernel_timing(self):
        ms = C.c_double(0)
        n = C.c_uint64(0)
        _check(lib().aqz_stage_kernel_timing(self.h, C.byref(ms), C.byref(n)), "timing")
        return ms.value, n.value

    def timing_mark(self, which):
        """Record timing event `which` (0 = begin, 1 = end) on the stage's
        stream, after everything enqueued so far."""
        _check(lib().aqz_stage_timing_mark(self.h, which), "timing_mark")

    def timing_elapsed(self):
        """ms between the begin and end marks (waits for the end mark)."""
        ms = C.c_double(0)
        _check(lib().aqz_stage_timing_elapsed(self.h, C.byref(ms)), "timing_elapsed")
        return ms.value

    def dominant_kernel(self):
        return lib().aqz_stage_dominant_kernel(self.h).decode()

    def zstd_far_ranges(self, level):
        """Ranges of the device zstd far pass over level's last compressed
        layer (aqz_stage_zstd_far_ranges; 0 = none ran)."""
        return lib().aqz_stage_zstd_far_ranges(self.h, level)

    def bind_host_thread(self):
        """aqz_stage_bind_host_thread: pin the calling thread to the CPUs of
        the device's NUMA node (memory it first touches lands there)."""
        _check(lib().aqz_stage_bind_host_thread(self.h), "bind_host_thread")

    def host_affinity(self):
        """(NUMA node of the device, CPUs the host pools are pinned to)."""
        node, n = C.c_int32(-1), C.c_uint32(0)
        _check(lib().aqz_stage_host_affinity(self.h, C.byref(node), C.byref(n)),
               "host_affinity")
        return node.value, n.value

    def placement(self):
        """Creation-time placement search (bench option placement_tries):
        {"candidates_ms": [...], "kept": i, "kept_ms_final", "reps", "mode",
        "peak_device_bytes", "probe_bus_gbs", "expected_ms", "alg_bytes",
        "accepted"} (empty candidate list when none ran)."""
        r = PlacementReportC()
        _check(lib().aqz_stage_placement_report(self.h, C.byref(r)), "placement_report")
        return {"candidates_ms": [round(r.ms[i], 5) for i in range(min(32, r.n))],
                "kept": r.kept, "kept_ms_final": round(r.kept_ms_final, 5),
                "reps": r.reps, "mode": r.mode,
                "peak_device_bytes": r.peak_device_bytes,
                "probe_bus_gbs": round(r.probe_bus_gbs, 1),
                "expected_ms": round(r.expected_ms, 5), "alg_bytes": r.alg_bytes,
                "accepted": bool(r.accepted),
                "stop": {1: "accepted", 2: "every try ran", 3: "no expectation (probe too small)",
                         4: "out of memory"}.get(r.stop, "no search"),
                "candidates_probe_gbs": [round(r.probe_gbs[i], 1)
                                         for i in range(min(32, r.n))]}

    # ---- device compression of resident layers ----------------------------
    def compress_layer(self, level, layer, codec=CODEC_BLOSC_LZ4, clevel=5, shuffle=1):
        c = CompressionC(codec, clevel, shuffle)
        _check(lib().aqz_stage_compress_layer(self.h, level, layer, C.byref(c)),
               "compress_layer")

    def compression_done(self, level, layer):
        d = C.c_int32(0)
        _check(lib().aqz_stage_compression_done(self.h, level, layer, C.byref(d)),
               "compression_done")
        return bool(d.value)

    def compressed_offsets(self, level, layer):
        n = self.layout(level)["chunks_per_layer"] + 1
        off = np.empty(n, dtype=np.uint64)
        _check(lib().aqz_stage_compressed_offsets(
            self.h, level, layer, off.ctypes.data_as(C.POINTER(C.c_uint64)), n),
            "compressed_offsets")
        return off

    def copy_compressed_async(self, level, layer, dst_ptr, cap):
        _check(lib().aqz_stage_copy_compressed_async(self.h, level, layer, dst_ptr, cap),
               "copy_compressed_async")

    def compressed_entries(self, level, layer):
        """[(chunk, shard, internal, offset, nbytes)] in output (shard-major) order."""
        n = self.layout(level)["chunks_per_layer"]
        arr = (ChunkEntryC * n)()
        _check(lib().aqz_stage_compressed_entries(self.h, level, layer, arr, n),
               "compressed_entries")
        return [(e.chunk, e.shard, e.internal, e.offset, e.nbytes) for e in arr]

    def shard_geometry(self, level):
        a, b, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
        _check(lib().aqz_stage_shard_geometry(self.h, level, C.byref(a), C.byref(b),
                                              C.byref(c)), "shard_geometry")
        return a.value, b.value, c.value

    def copy_compressed(self, level, layer):
        """(frames bytes, offsets) of a compressed layer, synchronously."""
        off = self.compressed_offsets(level, layer)
        out = np.empty(max(1, int(off[-1])), dtype=np.uint8)
        self.copy_compressed_async(level, layer, out.ctypes.data, out.nbytes)
        self.wait_copies()
        return out[:int(off[-1])], off


class Compressor:
    """blosc1/LZ4 frames of device-resident chunks (aqz_compressor_*)."""

    def __init__(self, chunk_bytes, typesize, codec=CODEC_BLOSC_LZ4, clevel=5, shuffle=1):
        c = CompressionC(codec, clevel, shuffle)
        h = C.c_void_p()
        _check(lib().aqz_compressor_create(chunk_bytes, typesize, C.byref(c), C.byref(h)),
               "aqz_compressor_create")
        self.h = h
        self.chunk_bytes = chunk_bytes

    def close(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.aqz_compressor_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    @property
    def blocksize(self):
        return lib().aqz_compressor_blocksize(self.h)

    def max_bytes(self, n_chunks):
        return lib().aqz_compressor_max_bytes(self.chunk_bytes, n_chunks)

    def run_ptr(self, chunks_ptr, pitch, n_chunks, dst_ptr, dst_cap, offsets_ptr,
                stream_ptr=None):
        _check(lib().aqz_compressor_run(self.h, chunks_ptr, pitch, n_chunks, dst_ptr,
                                        dst_cap, offsets_ptr, stream_ptr),
               "aqz_compressor_run")


def shard_table(offsets, extents) -> bytes:
    """Shard::write_table_ bytes (aqz_shard_table)."""
    n = len(offsets)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ext = np.ascontiguousarray(extents, dtype=np.uint64)
    out = np.empty(lib().aqz_shard_table_bytes(n), dtype=np.uint8)
    _check(lib().aqz_shard_table(off.ctypes.data, ext.ctypes.data, n, out.ctypes.data,
                                 out.nbytes), "aqz_shard_table")
    return out.tobytes()


def crc32c(data: bytes) -> int:
    return lib().aqz_crc32c(data, len(data))


class ShardAssembler:
    """zarr::Shard bookkeeping for one append-dimension shard row of a level
    (shard.cpp:55-166): each compressed layer's shard runs are appended at
    the shard's running offset, unwritten chunks keep the UINT64_MAX
    sentinel, and finalize() appends the index table + CRC-32C.  Host-side
    helper over the C ABI; the byte sink (file / S3) is the caller's."""

    def __init__(self, stage, level):
        self.cps, self.n_shards, self.lps = stage.shard_geometry(level)
        self.data = [bytearray() for _ in range(self.n_shards)]
        self.off = [[SHARD_UNWRITTEN] * self.cps for _ in range(self.n_shards)]
        self.ext = [[SHARD_UNWRITTEN] * self.cps for _ in range(self.n_shards)]

    def add_layer(self, frames, entries):
        for chunk, shard, internal, offset, nbytes in entries:
            if nbytes == 0:
                continue
            self.off[shard][internal] = len(self.data[shard])
            self.ext[shard][internal] = nbytes
            self.data[shard] += bytes(frames[offset:offset + nbytes])

    def finalize(self):
        return [bytes(self.data[s]) + shard_table(self.off[s], self.ext[s])
                for s in range(self.n_shards)]
