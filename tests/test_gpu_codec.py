"""GPU parity of the device chunk compressor (blosc1 + LZ4, SURVEY §8f
rank 2) through the C ABI.  The bar: every frame decodes -- with the
oracle's decoder and with c-blosc 1.21.0 -- to the chunk bytes exactly, the
header says what the reference's zarr.json promises (typesize, shuffle,
codec), chunks without data are skipped, and on camera-like data the
compression ratio stays close to c-blosc's own (compressed bytes are not
expected to match: block size and match finder differ by design)."""
import numpy as np
import pytest

from codec_helpers import (camera_like, chunk_payloads, header, libblosc,
                           libblosc_compress, libblosc_decode, oracle_decode)
from helpers import expected_stage_layers
from oracle_bindings import MEAN, SPACE, TIME, U16, synthetic_frames

pytestmark = pytest.mark.gpu

DT = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}


def _torch():
    import torch
    return torch


def compress_device(gpu, chunks: np.ndarray, ts, clevel=5, shuffle=1, pitch_pad=0):
    """chunks: (n, nbytes) uint8 host array -> list of frames (bytes)."""
    torch = _torch()
    n, nb = chunks.shape
    pitch = nb + pitch_pad
    src = torch.zeros(n * pitch + 16, dtype=torch.uint8, device="cuda")
    srcv = src[:n * pitch].view(n, pitch)
    srcv[:, :nb] = torch.from_numpy(chunks).to("cuda")
    comp = gpu.Compressor(nb, ts, clevel=clevel, shuffle=shuffle)
    cap = comp.max_bytes(n)
    dst = torch.empty(cap, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    comp.run_ptr(src.data_ptr(), pitch, n, dst.data_ptr(), cap, off.data_ptr(),
                 torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    o = off.cpu().numpy().astype(np.uint64)
    d = dst.cpu().numpy()
    frames = [d[int(o[i]):int(o[i + 1])].tobytes() for i in range(n)]
    bs = comp.blocksize
    comp.close()
    return frames, int(o[-1]), bs


def check_frames(frames, chunks, ts, shuffle, clevel):
    for i, fr in enumerate(frames):
        data = chunks[i].tobytes()
        h = header(fr)
        assert h["version"] == 2 and h["typesize"] == ts and h["nbytes"] == len(data)
        assert h["cbytes"] == len(fr)
        assert (h["flags"] >> 5) == 1                       # LZ4
        if not h["flags"] & 0x2:
            assert bool(h["flags"] & 0x1) == (shuffle == 1)
            assert bool(h["flags"] & 0x4) == (shuffle == 2)
        if clevel == 0:
            assert h["flags"] & 0x2
        assert len(fr) <= len(data) + 16
        assert oracle_decode(fr) == data, (i, h)
        if libblosc() is not None:
            assert libblosc_decode(fr) == data, (i, h)


@pytest.mark.parametrize("ts", [1, 2, 4, 8])
@pytest.mark.parametrize("shuffle", [0, 1, 2])
def test_compressor_decodes_exactly(gpu, ts, shuffle):
    rng = np.random.default_rng(10 * ts + shuffle)
    for n_px in (16384, 40_000 // ts * 3, 1000, 50):
        pay = chunk_payloads(rng, DT[ts], n_px)
        chunks = np.stack([a.view(np.uint8) for a in pay.values()])
        frames, total, _ = compress_device(gpu, chunks, ts, 5, shuffle)
        assert total == sum(len(f) for f in frames)
        check_frames(frames, chunks, ts, shuffle, 5)


def test_compressor_edge_sizes_and_pitch(gpu):
    rng = np.random.default_rng(3)
    # leftover blocks larger than one LDS stream, tiny chunks, odd sizes, a
    # chunk pitch above the chunk size
    for ts, n_px, pad in ((2, 16384 + 12000, 0), (4, 16384 * 2 + 9000, 48), (1, 13, 0),
                          (1, 12, 3), (2, 129, 0), (8, 127, 8), (1, 70_001, 16)):
        pay = chunk_payloads(rng, DT[ts], n_px, kinds=("camera", "random", "ramp"))
        chunks = np.stack([a.view(np.uint8) for a in pay.values()])
        for sh in (0, 1, 2):
            frames, _, _ = compress_device(gpu, chunks, ts, 5, sh, pitch_pad=pad)
            check_frames(frames, chunks, ts, sh, 5)


def test_compressor_clevel0_stores(gpu):
    rng = np.random.default_rng(4)
    chunks = np.stack([camera_like(rng, 20000, np.uint16).view(np.uint8) for _ in range(3)])
    frames, _, _ = compress_device(gpu, chunks, 2, 0, 1)
    check_frames(frames, chunks, 2, 1, 0)


@pytest.mark.skipif(libblosc() is None, reason="c-blosc not in this image")
def test_compression_ratio_close_to_cblosc(gpu):
    """Camera-like u16 chunks of the C2 layer shape (256x256x64): the device
    frames are at most 10% larger than c-blosc lz4 clevel 5's."""
    rng = np.random.default_rng(5)
    n_px = 256 * 256 * 8
    chunks = np.stack([camera_like(rng, n_px, np.uint16, noise=n).view(np.uint8)
                       for n in (3.0, 30.0)])
    for sh in (1, 2):
        frames, total, _ = compress_device(gpu, chunks, 2, 5, sh)
        check_frames(frames, chunks, 2, sh, 5)
        ref = sum(len(libblosc_compress(c.tobytes(), 2, 5, sh)) for c in chunks)
        assert total <= 1.10 * ref, (sh, total, ref)


def test_stage_compress_layer(gpu):
    """Stage hand-off with device compression: every chunk layer of every
    level compressed on the device, copied back, decoded == the oracle's
    chunk layer; chunks without data (an all-zero region) are skipped."""
    dims = [(TIME, 0, 2, 1), (SPACE, 512, 128, 1), (SPACE, 384, 128, 1)]
    n = 6
    frames = synthetic_frames(U16, n, 512, 384, 9)
    frames[:, :128, :] = 0          # one row of chunks without data
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    st = gpu.Stage(dims, U16, MEAN, layer_slots=2, max_batch_frames=2)
    L = st.n_levels()
    lay = [st.layout(l) for l in range(L)]
    got = {}
    for b in range(0, n, 2):
        st.append(np.ascontiguousarray(frames[b:b + 2]))
        for l in range(L):
            layer = st.frames_written(l) // lay[l]["frames_per_layer"] - 1
            if layer >= 0 and (l, layer) not in got:
                st.compress_layer(l, layer, clevel=5, shuffle=1)
                got[(l, layer)] = (st.copy_compressed(l, layer)[0],
                                   st.compressed_entries(l, layer))
    assert sorted(got) == sorted(exp)
    for (l, layer), (buf, flags) in exp.items():
        data, ent = got[(l, layer)]
        bpc = lay[l]["bytes_per_chunk"]
        assert sorted(e[0] for e in ent) == list(range(lay[l]["chunks_per_layer"]))
        for c, _, _, o, nb in ent:
            fr = data[o:o + nb].tobytes()
            if not flags[c]:
                assert len(fr) == 0, (l, layer, c)
                continue
            chunk = buf[c * bpc:(c + 1) * bpc].tobytes()
            assert oracle_decode(fr) == chunk, (l, layer, c)
    st.close()


def parse_shard(blob: bytes, cps: int):
    """(offsets, extents) of a shard file; checks the index CRC-32C."""
    import struct
    from codec_helpers import crc32c
    tbl = blob[len(blob) - 16 * cps - 4:]
    body, crc = tbl[:-4], struct.unpack("<I", tbl[-4:])[0]
    assert crc32c(body) == crc, "shard index checksum"
    pairs = [struct.unpack("<QQ", body[16 * i:16 * i + 16]) for i in range(cps)]
    return [p[0] for p in pairs], [p[1] for p in pairs]


def test_stage_shards_from_device_frames(gpu):
    """Shard packing: compressed layers leave the device
    shard-major; ShardAssembler appends each shard's run at its running
    offset over the layers of one append-dimension shard row and writes the
    index + CRC-32C.  Every written (offset, extent) decodes to the oracle's
    chunk at that internal index; chunks without data and the ragged edge
    shard's missing chunks carry the UINT64_MAX sentinel."""
    from oracle_bindings import OracleDims, OracleDownsampler
    # y: 4 chunks -> 2 shards; x: 3 chunks -> 2 shards (one ragged);
    # t: 2 layers per shard row
    dims = [(TIME, 0, 2, 2), (SPACE, 512, 128, 2), (SPACE, 384, 128, 2)]
    n = 8
    frames = synthetic_frames(U16, n, 512, 384, 21)
    frames[:, 128:256, :] = 0
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    ods = OracleDownsampler(dims, U16, MEAN, 0)
    st = gpu.Stage(dims, U16, MEAN, layer_slots=2, max_batch_frames=2)
    L = st.n_levels()
    lay = [st.layout(l) for l in range(L)]
    rows = {}   # (level, shard row) -> ShardAssembler
    done = {l: 0 for l in range(L)}
    for b in range(0, n, 2):
        st.append(np.ascontiguousarray(frames[b:b + 2]))
        for l in range(L):
            while done[l] < st.frames_written(l) // lay[l]["frames_per_layer"]:
                layer = done[l]
                st.compress_layer(l, layer, clevel=5, shuffle=2)
                data, _ = st.copy_compressed(l, layer)
                ent = st.compressed_entries(l, layer)
                lps = st.shard_geometry(l)[2]
                key = (l, layer // lps)
                if key not in rows:
                    rows[key] = gpu.ShardAssembler(st, l)
                rows[key].add_layer(data, ent)
                done[l] += 1
    st.close()
    checked = 0
    for (l, row), asm in rows.items():
        od = OracleDims(ods.level_dims(l), U16)
        cim = od.number_of_chunks_in_memory()
        bpc = od.bytes_per_chunk()
        blobs = asm.finalize()
        want = {}  # (shard, internal) -> chunk bytes or None (no data)
        for cl in range(asm.lps):
            layer = row * asm.lps + cl
            if (l, layer) not in exp:
                continue
            buf, flags = exp[(l, layer)]
            for c in range(cim):
                idx = cl * cim + c
                key = (od.shard_index_for_chunk(idx), od.shard_internal_index(idx))
                want[key] = buf[c * bpc:(c + 1) * bpc].tobytes() if flags[c] else None
        for s, blob in enumerate(blobs):
            offs, exts = parse_shard(blob, asm.cps)
            for i in range(asm.cps):
                w = want.get((s, i))
                if w is None:
                    assert offs[i] == gpu.SHARD_UNWRITTEN and exts[i] == gpu.SHARD_UNWRITTEN
                    continue
                fr = blob[offs[i]:offs[i] + exts[i]]
                assert oracle_decode(fr) == w, (l, row, s, i)
                checked += 1
    assert checked > 0


def test_compressed_handoff_pinned_and_pageable(gpu):
    """aqz_stage_copy_compressed_async into pinned memory of the codec bound
    (aqz_compressor_max_bytes) gives the same bytes as into pageable memory,
    for lz4, blosc-zstd and zstd, and writes nothing past the frames."""
    dims = [(TIME, 0, 4, 1), (SPACE, 256, 64, 1), (SPACE, 192, 64, 1)]
    frames = synthetic_frames(U16, 4, 256, 192, 12)
    frames[:, :64] = 0  # chunks without data
    for codec, shuffle in ((1, 1), (2, 2), (3, 0)):
        st = gpu.Stage(dims, U16, MEAN, layer_slots=2, max_batch_frames=4)
        st.append(np.ascontiguousarray(frames))
        lay = st.layout(0)
        st.compress_layer(0, 0, codec=codec, clevel=5, shuffle=shuffle)
        bound = gpu.lib().aqz_compressor_max_bytes(lay["bytes_per_chunk"],
                                                   lay["chunks_per_layer"])
        pinned = gpu.HostBuffer(bound)
        pinned.array[:] = 0xAB
        st.copy_compressed_async(0, 0, pinned.ptr, bound)
        st.wait_copies()
        ref, off = st.copy_compressed(0, 0)  # into pageable memory
        total = int(off[-1])
        assert total > 0
        assert np.array_equal(pinned.array[:total], ref), codec
        assert (pinned.array[total:total + 64] == 0xAB).all()  # nothing past the frames
        st.close()
