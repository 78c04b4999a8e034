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


def camera_like(rng, n_px: int, dtype, level=1000.0, noise=30.0) -> np.ndarray:
    """Smooth background + shot-noise-like jitter, the shape of sCMOS frames."""
    x = np.arange(n_px, dtype=np.float64)
    base = level + 200.0 * np.sin(x / 977.0)
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
