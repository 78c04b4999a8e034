"""The format pieces of the device zstd encoder (acquire-zarr_amd/csrc/
aqz_zstd.hh), checked on the CPU: tests/zstd/zstd_host.cpp runs the same
__host__ __device__ building blocks as a serial encoder over zeros, random,
camera-like (plain and byte-shuffled), sparse, skewed, wide-alphabet,
binary and text payloads from 0 B to 1 MiB, with and without LZ sequences,
and libzstd must decode every frame exactly -- the reference's own zstd
1.4.9 (conda) and the system's.  Every path is taken: RLE, raw and
compressed blocks, FSE-compressed and direct Huffman trees, Treeless
literals, predefined-FSE sequences."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from codec_helpers import libzstd, zstd_decode

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ZDIR = os.path.join(REPO, "tests", "zstd")
LIBS = [p for p in ("/opt/conda/lib/libzstd.so.1", "libzstd.so.1")
        if p == "libzstd.so.1" or os.path.exists(p)]


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-C", ZDIR], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return ZDIR


@pytest.mark.parametrize("lib", LIBS)
def test_format_pieces_decode_exactly(built, lib):
    r = subprocess.run([os.path.join(built, "zstd_host"), lib], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "decoded exactly" in r.stdout


@pytest.mark.skipif(libzstd() is None, reason="no libzstd")
def test_model_frames_through_ctypes(built):
    L = C.CDLL(os.path.join(built, "libzstd_host.so"))
    L.zh_encode_frame.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_void_p, C.c_uint64]
    L.zh_encode_frame.restype = C.c_uint64
    rng = np.random.default_rng(3)
    for n in (1, 777, 32768, 100003):
        for kind in range(3):
            src = {0: rng.integers(0, 256, n, dtype=np.uint8),
                   1: np.zeros(n, np.uint8),
                   2: (rng.normal(100, 4, n).clip(0, 255)).astype(np.uint8)}[kind]
            for lz in (0, 1):
                out = np.zeros(n + 4096, np.uint8)
                k = L.zh_encode_frame(src.ctypes.data, n, lz, out.ctypes.data, out.size)
                assert k > 0
                assert zstd_decode(out[:k].tobytes(), n) == src.tobytes()
