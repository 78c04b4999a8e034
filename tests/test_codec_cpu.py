"""CPU tests of the compression oracle (oracle/aqz_codec_oracle.c): it must
decode what c-blosc 1.21.0 itself writes, and c-blosc must decode frames
built with the oracle's byte shuffle / bitshuffle and the split rule --
which pins the frame layout the GPU compressor writes.  Plus CRC-32C known
answers (the shard index checksum, shard.cpp:145-166)."""
import struct

import numpy as np
import pytest

from codec_helpers import (chunk_payloads, crc32c, libblosc, libblosc_compress,
                           libblosc_decode, oracle_decode, shuffle)

needs_blosc = pytest.mark.skipif(libblosc() is None, reason="c-blosc not in this image")


def test_crc32c_known_answers():
    # RFC 3720 B.4 and the common check value
    assert crc32c(b"123456789") == 0xE3069283
    assert crc32c(bytes(32)) == 0x8A9136AA
    assert crc32c(bytes([0xFF] * 32)) == 0x62A8AB43
    assert crc32c(bytes(range(32))) == 0x46DD794E


@needs_blosc
@pytest.mark.parametrize("ts", [1, 2, 4, 8])
def test_oracle_decodes_cblosc_frames(ts):
    rng = np.random.default_rng(ts)
    dt = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[ts]
    for n_px in (50, 1000, 40_000, 70_001):
        for kind, a in chunk_payloads(rng, dt, n_px).items():
            data = a.tobytes()
            for clevel in (1, 5, 9):
                for sh in (0, 1, 2):
                    fr = libblosc_compress(data, ts, clevel, sh)
                    assert oracle_decode(fr) == data, (ts, n_px, kind, clevel, sh)


def _frame(data: bytes, ts: int, sh: int, bs: int) -> bytes:
    """A blosc1/LZ4 frame with every stream stored raw, shuffled by the oracle."""
    n = len(data)
    nfull, left = divmod(n, bs)
    nb = nfull + (1 if left else 0)
    off = 16 + 4 * nb
    starts, body = [], b""
    for j in range(nb):
        blk = data[j * bs:j * bs + (left if j == nfull else bs)]
        sb = shuffle("shuffle", ts, blk) if sh == 1 and ts > 1 else (
            shuffle("bitshuffle", ts, blk) if sh == 2 else blk)
        ns = ts if (ts <= 16 and len(blk) // ts >= 128 and j < nfull) else 1
        ne = len(blk) // ns
        starts.append(off)
        rec = b"".join(struct.pack("<I", ne) + sb[s * ne:(s + 1) * ne] for s in range(ns))
        body += rec
        off += len(rec)
    flags = 0x20 | (1 if sh == 1 else 0) | (4 if sh == 2 else 0)
    hdr = bytes([2, 1, flags, ts]) + struct.pack("<III", n, bs, 16 + 4 * nb + len(body))
    return hdr + b"".join(struct.pack("<I", s) for s in starts) + body


@needs_blosc
@pytest.mark.parametrize("ts", [1, 2, 4, 8])
@pytest.mark.parametrize("sh", [0, 1, 2])
def test_cblosc_decodes_oracle_shuffled_frames(ts, sh):
    rng = np.random.default_rng(100 * ts + sh)
    for n, bs in ((4096, 1024), (5000, 1024), (65536, 16384 * ts), (200, 64 * ts),
                  (3000, 72 * ts), (3000, 24 * ts)):
        n -= n % ts
        bs = min(bs, n)
        bs -= bs % ts
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        fr = _frame(data, ts, sh, bs)
        assert libblosc_decode(fr) == data, (n, bs)
        assert oracle_decode(fr) == data, (n, bs)


def test_shuffles_invert():
    rng = np.random.default_rng(7)
    for ts in (1, 2, 3, 4, 8):
        for n in (0, 7, 64, 1000, 4096 + 5):
            d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            assert shuffle("unshuffle", ts, shuffle("shuffle", ts, d)) == d
            assert shuffle("bitunshuffle", ts, shuffle("bitshuffle", ts, d)) == d


def test_shard_table_layout_and_crc():
    """aqz_shard_table (C ABI, host code) == Shard::write_table_ restated:
    (offset, extent) little-endian u64 pairs, UINT64_MAX for unwritten
    chunks, then CRC-32C of the pairs (shard.cpp:145-166)."""
    import aqz
    U = (1 << 64) - 1
    offsets = [0, U, 1000, 17, U]
    extents = [1000, U, 5, 983, U]
    t = aqz.shard_table(offsets, extents)
    body = b"".join(struct.pack("<QQ", o, e) for o, e in zip(offsets, extents))
    assert t[:-4] == body
    assert struct.unpack("<I", t[-4:])[0] == crc32c(body)
    assert aqz.crc32c(b"123456789") == 0xE3069283
    rng = np.random.default_rng(0)
    for n in (0, 1, 31, 1000):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert aqz.crc32c(d) == crc32c(d)


@pytest.mark.skipif(libblosc() is None, reason="c-blosc not in this image")
def test_blosc_zstd_decoder_restatement_pinned_to_cblosc():
    """codec_helpers.blosc_zstd_decode (the GPU zstd tests' independent
    decoder) reads c-blosc 1.21.0's own zstd frames -- split and unsplit
    blocks, byte/bit shuffle, raw (incompressible) streams, memcpyed frames."""
    from codec_helpers import blosc_zstd_decode, camera_like, libblosc_compress, libzstd
    if libzstd() is None:
        pytest.skip("no libzstd")
    rng = np.random.default_rng(1)
    for ts, dt in ((1, np.uint8), (2, np.uint16), (4, np.uint32), (8, np.uint64)):
        for sh in (0, 1, 2):
            for clevel in (0, 1, 5, 9):
                a = camera_like(rng, 300_000 // ts, dt).tobytes()
                assert blosc_zstd_decode(libblosc_compress(a, ts, clevel, sh, b"zstd")) == a
                r = rng.integers(0, 256, len(a), dtype=np.uint8).tobytes()
                assert blosc_zstd_decode(libblosc_compress(r, ts, clevel, sh, b"zstd")) == r
