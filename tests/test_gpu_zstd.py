"""GPU stage with the zstd codecs (SURVEY §8f rank 2 remainder): blosc1
frames with codec zstd (zarr.common.cpp:106-140 with "zstd") and plain zstd
frames (zarr.common.cpp:142-166), as Chunk::compress_and_take_buffer
dispatches them (chunk.cpp:78-106).  Two engines: the device encoder
(default; aqz_codec.hip zstd_* kernels over aqz_zstd.hh) and, with
AQZ_ZSTD_HOST=1, the device shuffle + host libzstd pool (aqz_hostzstd.hh).
The device frames are also compared byte for byte with the serial model of
the same encoder (tests/zstd/libzstd_host.so), which libzstd decodes on the
CPU suite.

Bar: every frame decodes to the oracle's chunk exactly -- blosc-zstd with a
restated blosc1 decoder over libzstd (codec_helpers.blosc_zstd_decode) and
with c-blosc 1.21.0 itself, plain zstd with libzstd -- chunks without data
are skipped, incompressible chunks become memcpyed frames (blosc's rule),
and the ratio on camera-like data stays close to c-blosc's zstd."""
import ctypes as C
import os

import numpy as np
import pytest

from codec_helpers import (blosc_zstd_decode, camera_like, header, libblosc,
                           libblosc_compress, libblosc_decode, libzstd, zstd_compress,
                           zstd_decode)
from helpers import expected_stage_layers
from oracle_bindings import F32, F64, MEAN, SPACE, TIME, U8, U16, synthetic_frames

pytestmark = pytest.mark.gpu

needs_zstd = pytest.mark.skipif(libzstd() is None, reason="no libzstd to decode with")
MODEL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "zstd", "libzstd_host.so")


@pytest.fixture(params=["device", "host"])
def engine(request, monkeypatch):
    monkeypatch.setenv("AQZ_ZSTD_HOST", "1" if request.param == "host" else "0")
    return request.param


def model_frame(data: bytes, lz: int = 0, glog2: int = 3) -> bytes:
    """The serial model's frame; glog2 = log2 of the zstd blocks per Huffman
    group (aqz_codec.hh zstd_huf_group_log2)."""
    L = C.CDLL(MODEL)
    L.zh_encode_frame_g.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_uint32, C.c_void_p,
                                    C.c_uint64]
    L.zh_encode_frame_g.restype = C.c_uint64
    src = np.frombuffer(data, np.uint8)
    out = np.zeros(len(data) + 4096, np.uint8)
    n = L.zh_encode_frame_g(src.ctypes.data, len(data), lz, glog2, out.ctypes.data, out.size)
    assert n > 0
    return out[:n].tobytes()


def _frames(dtype, n, h, w, seed):
    """Half incompressible (random) rows, half camera-like, and one band of
    all-zero chunks."""
    fr = synthetic_frames(dtype, n, h, w, seed)
    rng = np.random.default_rng(seed)
    npdt = fr.dtype
    cam = camera_like(rng, n * (h // 2) * w, np.uint16).astype(np.float64)
    if dtype == U8:
        cam = cam / 8
    fr[:, h // 2:, :] = cam.astype(npdt).reshape(n, h // 2, w)
    fr[:, : h // 8, :] = 0
    return fr


def _run(gpu, dtype, codec, clevel, shuffle):
    dims = [(TIME, 0, 2, 1), (SPACE, 512, 128, 1), (SPACE, 384, 128, 1)]
    n = 6
    frames = _frames(dtype, n, 512, 384, 40 + codec * 3 + shuffle)
    exp, fw, _ = expected_stage_layers(dims, dtype, MEAN, frames)
    st = gpu.Stage(dims, dtype, MEAN, layer_slots=2, max_batch_frames=2)
    L = st.n_levels()
    lay = [st.layout(l) for l in range(L)]
    got = {}
    for b in range(0, n, 2):
        st.append(np.ascontiguousarray(frames[b:b + 2]))
        for l in range(L):
            layer = st.frames_written(l) // lay[l]["frames_per_layer"] - 1
            if layer >= 0 and (l, layer) not in got:
                st.compress_layer(l, layer, codec=codec, clevel=clevel, shuffle=shuffle)
                got[(l, layer)] = (st.copy_compressed(l, layer)[0],
                                   st.compressed_entries(l, layer))
    st.close()
    assert sorted(got) == sorted(exp)
    n_memcpy = n_frames = 0
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
            n_frames += 1
            if codec == 3:
                assert zstd_decode(fr, bpc) == chunk, (l, layer, c)
                continue
            h = header(fr)
            assert h["version"] == 2 and (h["flags"] >> 5) == 4 and h["nbytes"] == bpc
            assert h["typesize"] == {U8: 1, U16: 2, F32: 4, F64: 8}[dtype]
            assert h["cbytes"] == len(fr) and len(fr) <= bpc + 16
            if h["flags"] & 0x2:
                n_memcpy += 1
            else:
                assert bool(h["flags"] & 0x1) == (shuffle == 1)
                assert bool(h["flags"] & 0x4) == (shuffle == 2)
            assert blosc_zstd_decode(fr) == chunk, (l, layer, c, h)
            if libblosc() is not None:
                assert libblosc_decode(fr) == chunk, (l, layer, c, h)
    assert n_frames > 0
    return n_memcpy


@needs_zstd
@pytest.mark.parametrize("dtype", [U8, U16, F32, F64], ids=["u8", "u16", "f32", "f64"])
@pytest.mark.parametrize("shuffle", [0, 1, 2])
def test_stage_blosc_zstd_layers(gpu, engine, dtype, shuffle):
    _run(gpu, dtype, 2, 5, shuffle)


# Device encoder bytes against the reference codecs on the same chunks
# (tools/zstd_lab.cpp models the encoder: per-64-KiB Huffman groups (one bit
# plane under bitshuffle), fitted segment sequence tables, a 12 KiB parse
# history at level >= 3, and from level 5 the far candidates of zstd_far --
# 5-byte coincidences anywhere earlier in the chunk, libzstd's 2 MiB-window
# matches on noisy data): blosc-zstd within 5% of c-blosc zstd clevel 5, plain
# zstd within 10% of libzstd level 5, on camera-like and dim data.
DEVICE_BOUND = {("camera", 2): 1.05, ("dim", 2): 1.05, ("camera", 3): 1.10, ("dim", 3): 1.10}


@needs_zstd
def test_stage_blosc_zstd_clevel0_memcpyed(gpu, engine):
    assert _run(gpu, U16, 2, 0, 1) > 0


@needs_zstd
@pytest.mark.parametrize("level", [1, 3, 9])
def test_stage_plain_zstd_layers(gpu, engine, level):
    _run(gpu, U16, 3, level, 0)


@needs_zstd
def test_plain_zstd_incompressible_large_chunks(gpu):
    """Incompressible 2 MiB chunks (BASELINE configs[0]'s 128x128x64 u16
    chunk): every plain zstd frame is raw blocks, one 3-byte header per
    8 KiB device block, so the layer stays within aqz_compressor_max_bytes
    (the device output buffer) and decodes exactly (regression: the bound
    once assumed 32 KiB blocks and the frames overran it)."""
    dims = [(TIME, 0, 64, 1), (SPACE, 256, 128, 2), (SPACE, 256, 128, 2)]
    frames = synthetic_frames(U16, 64, 256, 256, 77)
    exp, _, _ = expected_stage_layers(dims, U16, MEAN, frames)
    st = gpu.Stage(dims, U16, MEAN, layer_slots=1, max_batch_frames=64)
    st.append(np.ascontiguousarray(frames))
    st.compress_layer(0, 0, codec=3, clevel=1, shuffle=0)
    data, off = st.copy_compressed(0, 0)
    ent = st.compressed_entries(0, 0)
    lay = st.layout(0)
    bpc, n = lay["bytes_per_chunk"], lay["chunks_per_layer"]
    st.close()
    assert bpc == 2 << 20 and n == 4
    assert int(off[-1]) <= gpu.lib().aqz_compressor_max_bytes(bpc, n)
    assert int(off[-1]) > n * bpc  # raw blocks: the headers cost bytes
    buf, _ = exp[(0, 0)]
    for c, _, _, o, nb in ent:
        fr = data[o:o + nb].tobytes()
        assert zstd_decode(fr, bpc) == buf[c * bpc:(c + 1) * bpc].tobytes(), c


@needs_zstd
@pytest.mark.skipif(libblosc() is None, reason="c-blosc not in this image")
@pytest.mark.parametrize("payload", ["camera", "dim"])
def test_blosc_zstd_ratio_close_to_cblosc(gpu, engine, payload):
    """One C2-shaped chunk layer level (256x256 chunks, 8 frames) of u16
    camera-like (level 1000, noise 30) or dim sCMOS (level 100, noise 3)
    data: the host-engine frames are at most 10% larger than c-blosc zstd
    clevel 5 (ZSTD_compress level 5 for plain zstd) on the same chunks; the
    device encoder within DEVICE_BOUND."""
    dims = [(TIME, 0, 8, 1), (SPACE, 512, 256, 1), (SPACE, 512, 256, 1)]
    rng = np.random.default_rng(8)
    kw = {} if payload == "camera" else {"level": 100.0, "noise": 3.0, "amp": 0.0}
    frames = camera_like(rng, 8 * 512 * 512, np.uint16, **kw).reshape(8, 512, 512)
    st = gpu.Stage(dims, U16, MEAN, multiscale=False, layer_slots=2, max_batch_frames=8)
    st.append(frames)
    layer, _ = st.copy_layer(0, 0)
    bpc = st.layout(0)["bytes_per_chunk"]
    chunks = [layer[c * bpc:(c + 1) * bpc].tobytes() for c in range(4)]
    for codec, shuffle, ref in ((2, 1, lambda ch: libblosc_compress(ch, 2, 5, 1, b"zstd")),
                                (2, 2, lambda ch: libblosc_compress(ch, 2, 5, 2, b"zstd")),
                                (3, 0, lambda ch: zstd_compress(ch, 5))):
        st.compress_layer(0, 0, codec=codec, clevel=5, shuffle=shuffle)
        data, off = st.copy_compressed(0, 0)
        ours = int(off[-1])
        theirs = sum(len(ref(ch)) for ch in chunks)
        bound = 1.10 if engine == "host" else DEVICE_BOUND[(payload, codec)]
        print(f"{engine} {payload} codec {codec} shuffle {shuffle}: {ours} vs {theirs} "
              f"bytes ({ours / theirs:.3f}x)")
        assert ours <= bound * theirs, (codec, shuffle, ours, theirs)
    st.close()


@needs_zstd
@pytest.mark.parametrize("codec,shuffle", [(3, 0), (2, 1)])
def test_device_zstd_levels_differ(gpu, monkeypatch, codec, shuffle):
    """The plain zstd level chooses the parse history (level >= 3: 12 KiB,
    >= 7: 28 KiB): on dim sCMOS data a higher level finds more matches and
    writes fewer bytes.  blosc-zstd clevels >= 1 share one operating point
    (a history does not pay on shuffled planes).  Every level's frames decode
    exactly."""
    monkeypatch.setenv("AQZ_ZSTD_HOST", "0")
    dims = [(TIME, 0, 8, 1), (SPACE, 512, 256, 1), (SPACE, 512, 256, 1)]
    rng = np.random.default_rng(9)
    frames = camera_like(rng, 8 * 512 * 512, np.uint16, level=100.0, noise=3.0,
                         amp=0.0).reshape(8, 512, 512)
    st = gpu.Stage(dims, U16, MEAN, multiscale=False, layer_slots=2, max_batch_frames=8)
    st.append(frames)
    layer, _ = st.copy_layer(0, 0)
    bpc = st.layout(0)["bytes_per_chunk"]
    sizes = {}
    levels = (1, 3, 9) if codec == 3 else (1, 2, 5)
    for lv in levels:
        st.compress_layer(0, 0, codec=codec, clevel=lv, shuffle=shuffle)
        data, off = st.copy_compressed(0, 0)
        sizes[lv] = int(off[-1])
        for c, _, _, o, nb in st.compressed_entries(0, 0):
            fr = data[o:o + nb].tobytes()
            chunk = layer[c * bpc:(c + 1) * bpc].tobytes()
            got = zstd_decode(fr, bpc) if codec == 3 else blosc_zstd_decode(fr)
            assert got == chunk, (lv, c)
    st.close()
    print(f"codec {codec}: bytes by level {sizes}")
    lo, mid, hi = levels
    if codec == 3:
        assert sizes[hi] < sizes[mid] < sizes[lo]
    else:
        assert sizes[hi] == sizes[mid] == sizes[lo]


@needs_zstd
def test_device_blosc_zstd_bitshuffle_levels_differ(gpu, monkeypatch):
    """blosc-zstd with bitshuffle: clevel c is zstd level 2c - 1 and the
    level chooses the parse history (clevel 1: none; 5: 28 KiB, which reaches
    the previous bit plane of a u16 block): on camera-like data clevel 5
    writes fewer bytes than clevel 1.  Every frame decodes exactly."""
    monkeypatch.setenv("AQZ_ZSTD_HOST", "0")
    dims = [(TIME, 0, 8, 1), (SPACE, 512, 256, 1), (SPACE, 512, 256, 1)]
    rng = np.random.default_rng(10)
    frames = camera_like(rng, 8 * 512 * 512, np.uint16).reshape(8, 512, 512)
    st = gpu.Stage(dims, U16, MEAN, multiscale=False, layer_slots=2, max_batch_frames=8)
    st.append(frames)
    layer, _ = st.copy_layer(0, 0)
    bpc = st.layout(0)["bytes_per_chunk"]
    sizes = {}
    for lv in (1, 5):
        st.compress_layer(0, 0, codec=2, clevel=lv, shuffle=2)
        data, off = st.copy_compressed(0, 0)
        sizes[lv] = int(off[-1])
        for c, _, _, o, nb in st.compressed_entries(0, 0):
            got = blosc_zstd_decode(data[o:o + nb].tobytes())
            assert got == layer[c * bpc:(c + 1) * bpc].tobytes(), (lv, c)
    st.close()
    print(f"blosc-zstd bitshuffle: bytes by clevel {sizes}")
    assert sizes[5] < sizes[1]


@needs_zstd
@pytest.mark.skipif(not os.path.exists(MODEL), reason="tests/zstd not built")
@pytest.mark.parametrize("codec,shuffle,clevel", [(3, 0, 5), (2, 1, 5), (2, 2, 5), (2, 2, 7)])
def test_device_frames_equal_serial_model(gpu, monkeypatch, codec, shuffle, clevel):
    """Literal-only frames: the device encoder's bytes equal the serial
    model's (same Huffman construction, same block decisions), frame by
    frame -- plain zstd per chunk, blosc-zstd per record of a shuffled
    block."""
    monkeypatch.setenv("AQZ_ZSTD_HOST", "0")
    dims = [(TIME, 0, 4, 1), (SPACE, 512, 256, 1), (SPACE, 384, 128, 1)]
    frames = _frames(U16, 4, 512, 384, 77)
    st = gpu.Stage(dims, U16, MEAN, multiscale=False, layer_slots=2, max_batch_frames=4,
                   zstd_flags=gpu.ZSTD_LITERALS_ONLY)
    st.append(frames)
    layer, flags = st.copy_layer(0, 0)
    bpc = st.layout(0)["bytes_per_chunk"]
    st.compress_layer(0, 0, codec=codec, clevel=clevel, shuffle=shuffle)
    data, _ = st.copy_compressed(0, 0)
    ent = st.compressed_entries(0, 0)
    st.close()
    checked = 0
    for c, _, _, o, nb in ent:
        fr = data[o:o + nb].tobytes()
        if not flags[c]:
            continue
        chunk = layer[c * bpc:(c + 1) * bpc].tobytes()
        if codec == 3:  # unshuffled: Huffman groups of 32 blocks
            assert fr == model_frame(chunk, glog2=5), c
            checked += 1
            continue
        h = header(fr)
        if h["flags"] & 0x2:
            continue
        bs = h["blocksize"]
        nblk = -(-bpc // bs)
        for j in range(nblk):
            blk = chunk[j * bs:(j + 1) * bs]
            sh = shuffle_block(shuffle, 2, blk)
            start = int.from_bytes(fr[16 + 4 * j:20 + 4 * j], "little")
            cs = int.from_bytes(fr[start:start + 4], "little")
            rec = fr[start + 4:start + 4 + cs]
            if cs == len(blk):
                assert rec == sh, (c, j)
            else:
                # bitshuffle at clevel >= 7: a Huffman group is one bit plane;
                # no shuffle: 32 blocks
                glog2 = 5 if shuffle == 0 else 3
                while (shuffle == 2 and clevel >= 7 and glog2 > 0
                       and (8192 << glog2) > len(blk) // 16):
                    glog2 -= 1
                assert rec == model_frame(sh, glog2=glog2), (c, j)
            checked += 1
    assert checked > 0


def shuffle_block(kind, ts, blk):
    from codec_helpers import shuffle
    if kind == 0:
        return blk
    return shuffle({1: "shuffle", 2: "bitshuffle"}[kind], ts, blk)


@needs_zstd
@pytest.mark.parametrize("level", [3, 9])
def test_plain_zstd_far_candidates_large_chunks(gpu, monkeypatch, level):
    """Plain zstd at the far-candidate levels (zstd_far: 4 / 8 hash slices)
    on chunks of 16 MiB (tag bits 7) and 2 MiB, camera-like, dim and random
    bands: every frame decodes to its chunk, and the far pass pays (fewer
    bytes than level 1 on the same layer)."""
    monkeypatch.setenv("AQZ_ZSTD_HOST", "0")
    rng = np.random.default_rng(30 + level)
    for T, hw in ((8, 1024), (4, 512)):
        dims = [(TIME, 0, T, 1), (SPACE, 2 * hw, hw, 1), (SPACE, hw, hw, 1)]
        cam = camera_like(rng, T * 2 * hw * hw, np.uint16).reshape(T, 2 * hw, hw)
        dim = camera_like(rng, T * hw * hw, np.uint16, level=100.0, noise=3.0,
                          amp=0.0).reshape(T, hw, hw)
        frames = cam.copy()
        frames[:, hw:, :] = dim                                  # chunk 1: dim sCMOS
        frames[:, hw:hw + hw // 8, :] = rng.integers(0, 65535, (T, hw // 8, hw))  # random band
        st = gpu.Stage(dims, U16, MEAN, multiscale=False, layer_slots=2, max_batch_frames=T)
        st.append(np.ascontiguousarray(frames))
        layer, _ = st.copy_layer(0, 0)
        bpc = st.layout(0)["bytes_per_chunk"]
        assert bpc == T * hw * hw * 2
        sizes = {}
        for lv in (1, level):
            st.compress_layer(0, 0, codec=3, clevel=lv, shuffle=0)
            data, off = st.copy_compressed(0, 0)
            sizes[lv] = int(off[-1])
            for c, _, _, o, nb in st.compressed_entries(0, 0):
                assert zstd_decode(data[o:o + nb].tobytes(), bpc) == \
                    layer[c * bpc:(c + 1) * bpc].tobytes(), (T, lv, c)
        st.close()
        print(f"{bpc >> 20} MiB chunks: bytes by level {sizes}")
        assert sizes[level] < sizes[1]


@needs_zstd
def test_plain_zstd_far_ranges_keep_the_bytes(gpu, monkeypatch):
    """A layer of one 16 MiB chunk (8 planes of 1024 x 1024 u16, dim sCMOS
    frames that repeat from plane to plane) at level 3: the far pass walks
    it in parallel ranges, each warmed up with the 1 MiB and two planes
    before it.  Against the single-range walk (zstd_flags bit 21): both
    decode, and the ranged frames are within 0.5% of its bytes."""
    monkeypatch.setenv("AQZ_ZSTD_HOST", "0")
    rng = np.random.default_rng(77)
    T, hw = 8, 1024
    base = camera_like(rng, hw * hw, np.uint16, level=100.0, noise=3.0, amp=20.0)
    frames = np.stack([base + rng.integers(0, 2, hw * hw).astype(np.uint16) * (t % 2)
                       for t in range(T)]).reshape(T, hw, hw)
    dims = [(TIME, 0, T, 1), (SPACE, hw, hw, 1), (SPACE, hw, hw, 1)]
    sizes, ranges = {}, {}
    for name, flags in (("ranges", 0), ("one", gpu.ZSTD_FAR_ONE_RANGE)):
        st = gpu.Stage(dims, U16, MEAN, multiscale=False, layer_slots=2, max_batch_frames=T,
                       zstd_flags=flags)
        st.append(np.ascontiguousarray(frames))
        layer, _ = st.copy_layer(0, 0)
        bpc = st.layout(0)["bytes_per_chunk"]
        st.compress_layer(0, 0, codec=3, clevel=3, shuffle=0)
        data, off = st.copy_compressed(0, 0)
        for c, _, _, o, nb in st.compressed_entries(0, 0):
            assert zstd_decode(data[o:o + nb].tobytes(), bpc) == \
                layer[c * bpc:(c + 1) * bpc].tobytes(), (name, c)
        sizes[name] = int(off[-1])
        ranges[name] = st.zstd_far_ranges(0)
        st.close()
    print(f"16 MiB chunk at level 3: bytes {sizes}, far ranges {ranges}")
    # the ranged walk ran, the A/B switch kept one range
    assert ranges["one"] == 1 and ranges["ranges"] > 1, ranges
    assert sizes["ranges"] <= 1.005 * sizes["one"], sizes


@needs_zstd
def test_plain_zstd_far_unaligned_chunks(gpu, monkeypatch):
    """u8 chunks of an odd byte count (3 x 127 x 129): the far pass needs
    4-byte aligned segments and is skipped; level 3 still decodes."""
    monkeypatch.setenv("AQZ_ZSTD_HOST", "0")
    dims = [(TIME, 0, 3, 1), (SPACE, 254, 127, 1), (SPACE, 258, 129, 1)]
    frames = _frames(U8, 3, 254, 258, 91)
    st = gpu.Stage(dims, U8, MEAN, multiscale=False, layer_slots=2, max_batch_frames=3)
    st.append(frames)
    layer, flags = st.copy_layer(0, 0)
    bpc = st.layout(0)["bytes_per_chunk"]
    assert bpc % 4 != 0
    st.compress_layer(0, 0, codec=3, clevel=3, shuffle=0)
    data, _ = st.copy_compressed(0, 0)
    for c, _, _, o, nb in st.compressed_entries(0, 0):
        if flags[c]:
            assert zstd_decode(data[o:o + nb].tobytes(), bpc) == \
                layer[c * bpc:(c + 1) * bpc].tobytes(), c
    st.close()
