"""ctypes bindings for the CPU oracle (oracle/liboracle.so) and, where it was
built, the compiled reference (oracle/_ref/libaqzref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")
REF_SO = os.path.join(ORACLE_DIR, "_ref", "libaqzref.so")

U8, U16, U32, U64, I8, I16, I32, I64, F32, F64 = range(10)
DECIMATE, MEAN, MIN, MAX = range(4)
SPACE, CHANNEL, TIME, OTHER = range(4)

NP_DTYPES = {
    U8: np.uint8, U16: np.uint16, U32: np.uint32, U64: np.uint64,
    I8: np.int8, I16: np.int16, I32: np.int32, I64: np.int64,
    F32: np.float32, F64: np.float64,
}
DTYPE_NAMES = {U8: "u8", U16: "u16", U32: "u32", U64: "u64", I8: "i8",
               I16: "i16", I32: "i32", I64: "i64", F32: "f32", F64: "f64"}
METHOD_NAMES = {DECIMATE: "decimate", MEAN: "mean", MIN: "min", MAX: "max"}


class Dim(C.Structure):
    _fields_ = [("type", C.c_int32), ("array_size_px", C.c_uint32),
                ("chunk_size_px", C.c_uint32),
                ("shard_size_chunks", C.c_uint32)]


def dims_array(dims):
    """dims: list of (type, array, chunk, shard) tuples."""
    arr = (Dim * len(dims))()
    for i, d in enumerate(dims):
        arr[i] = Dim(*d)
    return arr


def ensure_oracle_built() -> None:
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", ORACLE_DIR, "liboracle.so"], check=True,
                       stdout=subprocess.DEVNULL)


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        ensure_oracle_built()
        L = C.CDLL(ORACLE_SO)
        vp, sz, u32, u64, i32 = C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_int
        D = C.POINTER(Dim)
        L.or_scale_image.argtypes = [i32, i32, vp, sz, sz, vp]
        L.or_average_two_frames.argtypes = [i32, i32, vp, vp, sz]
        L.or_make_levels.argtypes = [D, i32, u32, C.POINTER(C.c_int), D, i32]
        L.or_chunk_lattice_index.argtypes = [D, i32, u64, i32]
        L.or_chunk_lattice_index.restype = u32
        L.or_tile_group_offset.argtypes = [D, i32, u64]
        L.or_tile_group_offset.restype = u32
        L.or_chunk_internal_offset.argtypes = [D, i32, i32, u64]
        L.or_chunk_internal_offset.restype = u64
        L.or_bytes_per_chunk.argtypes = [D, i32, i32]
        L.or_bytes_per_chunk.restype = u64
        L.or_number_of_chunks_in_memory.argtypes = [D, i32]
        L.or_number_of_chunks_in_memory.restype = u32
        L.or_frames_per_chunk_layer.argtypes = [D, i32]
        L.or_frames_per_chunk_layer.restype = u64
        L.or_shard_index_for_chunk.argtypes = [D, i32, u32]
        L.or_shard_index_for_chunk.restype = u32
        L.or_shard_internal_index.argtypes = [D, i32, u32]
        L.or_shard_internal_index.restype = u32
        L.or_write_frame_to_chunks.argtypes = [D, i32, i32, u64, vp, vp, vp]
        L.or_write_frame_to_chunks.restype = sz
        L.or_ds_create.argtypes = [D, i32, i32, i32, u32]
        L.or_ds_create.restype = vp
        L.or_ds_destroy.argtypes = [vp]
        L.or_ds_n_levels.argtypes = [vp]
        L.or_ds_level_dims.argtypes = [vp, i32]
        L.or_ds_level_dims.restype = D
        L.or_ds_add_frame.argtypes = [vp, vp, sz]
        L.or_ds_take_frame.argtypes = [vp, i32, vp, sz, C.POINTER(sz)]
        L.or_fill_splitmix.argtypes = [vp, sz, u64]
        _lib = L
    return _lib


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def ref():
    global _ref
    if _ref is None:
        L = C.CDLL(REF_SO)
        vp, sz, u32, u64, i32 = C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_int
        D = C.POINTER(Dim)
        L.ref_ds_create.argtypes = [D, i32, i32, i32, u32]
        L.ref_ds_create.restype = vp
        L.ref_ds_destroy.argtypes = [vp]
        L.ref_ds_n_levels.argtypes = [vp]
        L.ref_ds_level_dims.argtypes = [vp, i32, D, i32]
        L.ref_ds_add_frame.argtypes = [vp, vp, sz]
        L.ref_ds_take_frame.argtypes = [vp, i32, vp, sz, C.POINTER(sz)]
        L.ref_dims_create.argtypes = [D, i32, i32]
        L.ref_dims_create.restype = vp
        L.ref_dims_create_ordered.argtypes = [D, i32, i32, C.POINTER(sz)]
        L.ref_dims_create_ordered.restype = vp
        L.ref_dims_transpose_frame_id.argtypes = [vp, u64]
        L.ref_dims_transpose_frame_id.restype = u64
        L.ref_dims_destroy.argtypes = [vp]
        for name, rt, extra in [
            ("tile_group_offset", u32, [u64]),
            ("chunk_internal_offset", u64, [u64]),
            ("chunk_lattice_index", u32, [u64, u32]),
            ("bytes_per_chunk", u64, []),
            ("number_of_chunks_in_memory", u32, []),
            ("frames_per_chunk_layer", u64, []),
            ("shard_index_for_chunk", u32, [u32]),
            ("shard_internal_index", u32, [u32]),
        ]:
            f = getattr(L, "ref_dims_" + name)
            f.argtypes = [vp] + extra
            f.restype = rt
        L.ref_write_frame_to_chunks.argtypes = [vp, i32, u64, vp, vp, vp]
        L.ref_write_frame_to_chunks.restype = sz
        _ref = L
    return _ref


# ---------------------------------------------------------------------------
# numpy helpers
# ---------------------------------------------------------------------------
def splitmix_bytes(nbytes: int, seed: int) -> np.ndarray:
    """splitmix64 byte stream (same stream as or_fill_splitmix), vectorised."""
    n64 = (nbytes + 7) // 8
    M = (1 << 64) - 1
    with np.errstate(over="ignore"):
        idx = np.arange(1, n64 + 1, dtype=np.uint64)
        z = (np.uint64(seed & M) + idx * np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:nbytes].copy()


def synthetic_frames(dtype: int, n: int, h: int, w: int, seed: int) -> np.ndarray:
    """Fixed-seed frames: integer dtypes full range, float uniform [0, 65535]."""
    npdt = NP_DTYPES[dtype]
    if dtype in (F32, F64):
        raw = splitmix_bytes(n * h * w * 8, seed).view(np.uint64)
        vals = (raw >> np.uint64(11)).astype(np.float64) / float(1 << 53) * 65535.0
        return vals.astype(npdt).reshape(n, h, w)
    isz = np.dtype(npdt).itemsize
    return splitmix_bytes(n * h * w * isz, seed).view(npdt).reshape(n, h, w)


class OracleDownsampler:
    """zarr::Downsampler semantics on the C restatement (or the real
    reference with use_ref=True)."""

    def __init__(self, dims, dtype, method, max_levels=0, use_ref=False):
        self.use_ref = use_ref
        self.L = ref() if use_ref else lib()
        self.dtype = dtype
        self.dims = list(dims)
        d = dims_array(dims)
        if use_ref:
            self.h = self.L.ref_ds_create(d, len(dims), dtype, method, max_levels)
        else:
            self.h = self.L.or_ds_create(d, len(dims), dtype, method, max_levels)
        if not self.h:
            raise RuntimeError("downsampler create failed")

    def __del__(self):
        if getattr(self, "h", None):
            (self.L.ref_ds_destroy if self.use_ref else self.L.or_ds_destroy)(self.h)
            self.h = None

    def n_levels(self) -> int:
        return (self.L.ref_ds_n_levels if self.use_ref else self.L.or_ds_n_levels)(self.h)

    def level_dims(self, level):
        if self.use_ref:
            out = (Dim * 16)()
            n = self.L.ref_ds_level_dims(self.h, level, out, 16)
            return [(out[i].type, out[i].array_size_px, out[i].chunk_size_px,
                     out[i].shard_size_chunks) for i in range(n)]
        p = self.L.or_ds_level_dims(self.h, level)
        return [(p[i].type, p[i].array_size_px, p[i].chunk_size_px,
                 p[i].shard_size_chunks) for i in range(len(self.dims))]

    def add_frame(self, frame: np.ndarray) -> None:
        frame = np.ascontiguousarray(frame)
        f = self.L.ref_ds_add_frame if self.use_ref else self.L.or_ds_add_frame
        rc = f(self.h, frame.ctypes.data, frame.nbytes)
        if rc != 0:
            raise RuntimeError(f"add_frame failed rc={rc}")

    def take_frame(self, level):
        d = self.level_dims(level)
        h, w = d[-2][1], d[-1][1]
        out = np.empty((h, w), dtype=NP_DTYPES[self.dtype])
        nb = C.c_size_t(0)
        f = self.L.ref_ds_take_frame if self.use_ref else self.L.or_ds_take_frame
        if not f(self.h, level, out.ctypes.data, out.nbytes, C.byref(nb)):
            return None
        assert nb.value == out.nbytes, (nb.value, out.nbytes)
        return out


def oracle_scale_image(img: np.ndarray, dtype: int, method: int) -> np.ndarray:
    h, w = img.shape
    out = np.empty(((h + 1) // 2, (w + 1) // 2), dtype=img.dtype)
    img = np.ascontiguousarray(img)
    rc = lib().or_scale_image(dtype, method, img.ctypes.data, w, h, out.ctypes.data)
    assert rc == 0
    return out


def oracle_average_two(dst: np.ndarray, src: np.ndarray, dtype: int, method: int):
    dst = np.ascontiguousarray(dst).copy()
    src = np.ascontiguousarray(src)
    rc = lib().or_average_two_frames(dtype, method, dst.ctypes.data, src.ctypes.data, dst.size)
    assert rc == 0
    return dst


class OracleDims:
    """ArrayDimensions index math on the C restatement or the reference."""

    def __init__(self, dims, dtype, use_ref=False, order=None):
        self.dims = list(dims)
        self.dtype = dtype
        self.use_ref = use_ref
        self._d = dims_array(dims)
        self.n = len(dims)
        if use_ref:
            self.L = ref()
            if order is None:
                self.h = self.L.ref_dims_create(self._d, self.n, dtype)
            else:
                self._o = (C.c_size_t * len(order))(*order)
                self.h = self.L.ref_dims_create_ordered(self._d, self.n, dtype, self._o)
            assert self.h
        else:
            assert order is None, "the C oracle takes storage-order dims"
            self.L = lib()

    def __del__(self):
        if self.use_ref and getattr(self, "h", None):
            self.L.ref_dims_destroy(self.h)
            self.h = None

    def transpose_frame_id(self, fid):
        assert self.use_ref
        return self.L.ref_dims_transpose_frame_id(self.h, fid)

    def tile_group_offset(self, fid):
        if self.use_ref:
            return self.L.ref_dims_tile_group_offset(self.h, fid)
        return self.L.or_tile_group_offset(self._d, self.n, fid)

    def chunk_internal_offset(self, fid):
        if self.use_ref:
            return self.L.ref_dims_chunk_internal_offset(self.h, fid)
        return self.L.or_chunk_internal_offset(self._d, self.n, self.dtype, fid)

    def chunk_lattice_index(self, fid, dim):
        if self.use_ref:
            return self.L.ref_dims_chunk_lattice_index(self.h, fid, dim)
        return self.L.or_chunk_lattice_index(self._d, self.n, fid, dim)

    def bytes_per_chunk(self):
        if self.use_ref:
            return self.L.ref_dims_bytes_per_chunk(self.h)
        return self.L.or_bytes_per_chunk(self._d, self.n, self.dtype)

    def number_of_chunks_in_memory(self):
        if self.use_ref:
            return self.L.ref_dims_number_of_chunks_in_memory(self.h)
        return self.L.or_number_of_chunks_in_memory(self._d, self.n)

    def frames_per_chunk_layer(self):
        if self.use_ref:
            return self.L.ref_dims_frames_per_chunk_layer(self.h)
        return self.L.or_frames_per_chunk_layer(self._d, self.n)

    def shard_index_for_chunk(self, c):
        if self.use_ref:
            return self.L.ref_dims_shard_index_for_chunk(self.h, c)
        return self.L.or_shard_index_for_chunk(self._d, self.n, c)

    def shard_internal_index(self, c):
        if self.use_ref:
            return self.L.ref_dims_shard_internal_index(self.h, c)
        return self.L.or_shard_internal_index(self._d, self.n, c)

    def new_layer(self):
        nbytes = self.bytes_per_chunk() * self.number_of_chunks_in_memory()
        return (np.zeros(nbytes, dtype=np.uint8),
                np.zeros(self.number_of_chunks_in_memory(), dtype=np.uint8))

    def write_frame_to_chunks(self, fid, frame, layer, has_data):
        frame = np.ascontiguousarray(frame)
        if self.use_ref:
            return self.L.ref_write_frame_to_chunks(
                self.h, self.dtype, fid, frame.ctypes.data, layer.ctypes.data,
                has_data.ctypes.data)
        return self.L.or_write_frame_to_chunks(
            self._d, self.n, self.dtype, fid, frame.ctypes.data,
            layer.ctypes.data, has_data.ctypes.data)
