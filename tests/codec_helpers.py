"""Chunk-compression test helpers: the oracle's blosc1/LZ4 decoder and
shuffles (oracle/aqz_codec_oracle.c) and, where the image has it, c-blosc
1.21.0 itself (/opt/conda, copied into oracle/_ref/lib by `make -C oracle
ref`) as a second, independent decoder and as the ratio yardstick.

TEST INFRASTRUCTURE ONLY.
"""
from __future__ import annotations

import ctypes as C
import os
import struct

import numpy as np

from oracle_bindings import ORACLE_DIR, lib as oracle_lib

_LIBBLOSC_PATHS = (os.path.join(ORACLE_DIR, "_ref", "lib", "libblosc.so.1"),
                   "/opt/conda/lib/libblosc.so.1")
_blosc = None
_setup = False


def _oracle():
    global _setup
    L = oracle_lib()
    if not _setup:
        vp, sz = C.c_void_p, C.c_size_t
        L.or_blosc_decompress.argtypes = [vp, sz, vp, sz, vp]
        L.or_blosc_decompress.restype = C.c_long
        L.or_crc32c.argtypes = [vp, sz]
        L.or_crc32c.restype = C.c_uint32
        for f in ("or_shuffle", "or_unshuffle", "or_bitshuffle", "or_bitunshuffle"):
            getattr(L, f).argtypes = [sz, sz, vp, vp]
        L.or_lz4_decompress.argtypes = [vp, sz, vp, sz]
        L.or_lz4_decompress.restype = C.c_long
        _setup = True
    return L


def libblosc():
    """c-blosc 1.21.0 (test-only checker) or None when the image lacks it."""
    global _blosc
    if _blosc is None:
        for p in _LIBBLOSC_PATHS:
            if os.path.exists(p):
                L = C.CDLL(p)
                L.blosc_compress_ctx.argtypes = [C.c_int, C.c_int, C.c_size_t, C.c_size_t,
                                                 C.c_void_p, C.c_void_p, C.c_size_t,
                                                 C.c_char_p, C.c_size_t, C.c_int]
                L.blosc_decompress_ctx.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t,
                                                   C.c_int]
                _blosc = L
                break
        else:
            _blosc = False
    return _blosc or None


def header(frame: bytes):
    ver, verlz, flags, ts = frame[0], frame[1], frame[2], frame[3]
    nbytes, blocksize, cbytes = struct.unpack("<III", frame[4:16])
    return dict(version=ver, versionlz=verlz, flags=flags, typesize=ts,
                nbytes=nbytes, blocksize=blocksize, cbytes=cbytes)


def oracle_decode(frame) -> bytes:
    frame = bytes(frame)
    h = header(frame)
    out = C.create_string_buffer(max(1, h["nbytes"]))
    tmp = C.create_string_buffer(max(1, h["blocksize"], h["nbytes"]))
    r = _oracle().or_blosc_decompress(frame, len(frame), out, h["nbytes"], tmp)
    assert r == h["nbytes"], f"oracle blosc decode failed ({r})"
    return out.raw[:h["nbytes"]]


def libblosc_decode(frame) -> bytes:
    L = libblosc()
    frame = bytes(frame)
    h = header(frame)
    out = C.create_string_buffer(max(1, h["nbytes"]))
    r = L.blosc_decompress_ctx(frame, out, h["nbytes"], 1)
    assert r == h["nbytes"], f"c-blosc decode failed ({r})"
    return out.raw[:h["nbytes"]]


def libblosc_compress(data: bytes, typesize: int, clevel: int, shuffle: int,
                      cname: bytes = b"lz4") -> bytes:
    L = libblosc()
    out = C.create_string_buffer(len(data) + 16)
    n = L.blosc_compress_ctx(clevel, shuffle, typesize, len(data), data, out,
                             len(data) + 16, cname, 0, 1)
    assert n > 0
    return out.raw[:n]


def crc32c(data: bytes) -> int:
    return _oracle().or_crc32c(data, len(data))


def shuffle(kind: str, ts: int, data: bytes) -> bytes:
    out = C.create_string_buffer(max(1, len(data)))
    getattr(_oracle(), "or_" + kind)(ts, len(data), data, out)
    return out.raw[:len(data)]


def camera_like(rng, n_px: int, dtype, level=1000.0, noise=30.0, amp=200.0) -> np.ndarray:
    """Smooth background + shot-noise-like jitter, the shape of sCMOS frames
    (level 100, noise 3, amp 0: a dim low-light sCMOS frame)."""
    x = np.arange(n_px, dtype=np.float64)
    base = level + amp * np.sin(x / 977.0)
    v = base + rng.normal(0.0, noise, n_px)
    info = np.iinfo(dtype) if np.issubdtype(dtype, np.integer) else None
    if info is not None:
        v = np.clip(v, info.min, info.max)
    return v.astype(dtype)


def chunk_payloads(rng, dtype, n_px: int, kinds=("camera", "zeros", "random",
                                                  "sparse", "ramp")):
    out = {}
    nbytes = n_px * np.dtype(dtype).itemsize
    for k in kinds:
        if k == "camera":
            a = camera_like(rng, n_px, dtype)
        elif k == "zeros":
            a = np.zeros(n_px, dtype)
        elif k == "random":
            a = np.frombuffer(rng.integers(0, 256, nbytes, dtype=np.uint8).tobytes(),
                              dtype=dtype).copy()
        elif k == "sparse":
            a = np.zeros(n_px, dtype)
            idx = rng.integers(0, n_px, max(1, n_px // 50))
            a[idx] = 7
        else:
            a = (np.arange(n_px) % 251).astype(dtype)
        out[k] = a
    return out


# ---- zstd (blosc-zstd and plain zstd frames) ------------------------------
# the process's libzstd.so.1 first: PyTorch's HIP runtime (pre-loaded
# RTLD_GLOBAL by aqz) already holds the system copy, and a second copy of
# the same soname opened by path binds its internal calls to the first one
# (ZSTD_compress then frees with the wrong struct layout); the reference's
# 1.4.9 (conda) when no copy is loaded yet
_LIBZSTD_PATHS = ("libzstd.so.1", os.path.join(ORACLE_DIR, "_ref", "lib", "libzstd.so.1"),
                  "/opt/conda/lib/libzstd.so.1")
_zstd = None


def libzstd():
    """libzstd (test-only decoder): conda's copy, else the system's."""
    global _zstd
    if _zstd is None:
        for p in _LIBZSTD_PATHS:
            try:
                L = C.CDLL(p)
            except OSError:
                continue
            L.ZSTD_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
            L.ZSTD_decompress.restype = C.c_size_t
            L.ZSTD_isError.argtypes = [C.c_size_t]
            L.ZSTD_isError.restype = C.c_uint
            L.ZSTD_getFrameContentSize.argtypes = [C.c_void_p, C.c_size_t]
            L.ZSTD_getFrameContentSize.restype = C.c_ulonglong
            L.ZSTD_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                        C.c_int]
            L.ZSTD_compress.restype = C.c_size_t
            L.ZSTD_compressBound.argtypes = [C.c_size_t]
            L.ZSTD_compressBound.restype = C.c_size_t
            _zstd = L
            break
        else:
            _zstd = False
    return _zstd or None


def zstd_decode(frame, nbytes: int) -> bytes:
    L = libzstd()
    frame = bytes(frame)
    out = C.create_string_buffer(max(1, nbytes))
    n = L.ZSTD_decompress(out, nbytes, frame, len(frame))
    assert not L.ZSTD_isError(n) and n == nbytes, f"zstd decode failed ({n})"
    return out.raw[:nbytes]


def zstd_compress(data: bytes, level: int) -> bytes:
    L = libzstd()
    cap = L.ZSTD_compressBound(len(data))
    out = C.create_string_buffer(cap)
    n = L.ZSTD_compress(out, cap, data, len(data), level)
    assert not L.ZSTD_isError(n)
    return out.raw[:n]


def blosc_zstd_decode(frame) -> bytes:
    """A blosc1 frame decoded by this restatement of the published format
    (header, block starts, per block per stream (csize, bytes); csize ==
    stream bytes = stored raw) with libzstd for the streams and the oracle's
    unshuffles -- independent of c-blosc."""
    frame = bytes(frame)
    h = header(frame)
    nbytes, bs, ts, fl = h["nbytes"], h["blocksize"], h["typesize"], h["flags"]
    assert (fl >> 5) == 4, "not a zstd blosc frame"
    if fl & 0x2:
        return frame[16:16 + nbytes]
    nblocks = -(-nbytes // bs)
    starts = struct.unpack("<%dI" % nblocks, frame[16:16 + 4 * nblocks])
    out = bytearray()
    for j in range(nblocks):
        blen = min(bs, nbytes - j * bs)
        split = not (fl & 0x10) and ts <= 16 and blen // ts >= 128 and blen == bs
        ns = ts if split else 1
        pos = starts[j]
        blk = bytearray()
        for _ in range(ns):
            cs = struct.unpack("<I", frame[pos:pos + 4])[0]
            slen = blen // ns
            data = frame[pos + 4:pos + 4 + cs]
            blk += data if cs == slen else zstd_decode(data, slen)
            pos += 4 + cs
        if fl & 0x1 and ts > 1:
            blk = shuffle("unshuffle", ts, bytes(blk))
        elif fl & 0x4:
            blk = shuffle("bitunshuffle", ts, bytes(blk))
        out += blk
    return bytes(out)
