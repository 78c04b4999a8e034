"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Every test here runs the MI355X kernels via include/aqz_gpu.h and compares
with the oracle restatement (oracle/aqz_oracle.c), which the CPU suite pins
to the compiled reference and to tests/golden/.  Bar: bit-exact for integer
dtypes; floats bit-exact on every non-NaN value with NaN positions equal.
"""
import numpy as np
import pytest

from helpers import (assert_same_pixels, expected_stage_layers, oracle_cascade,
                     with_specials)
from oracle_bindings import (CHANNEL, DECIMATE, DTYPE_NAMES, F32, F64, I8,
                             I16, I32, I64, MAX, MEAN, METHOD_NAMES, MIN, SPACE,
                             TIME, U8, U16, U32, U64, NP_DTYPES, synthetic_frames)

pytestmark = pytest.mark.gpu

ALL_DTYPES = [U8, U16, U32, U64, I8, I16, I32, I64, F32, F64]
ALL_METHODS = [DECIMATE, MEAN, MIN, MAX]
SHAPES = [(2, 2), (3, 3), (5, 7), (11, 11), (37, 29), (64, 48), (130, 67)]


def _frames(dtype, n, h, w, seed, specials=True):
    fr = synthetic_frames(dtype, n, h, w, seed)
    if specials:
        fr = with_specials(fr, dtype, seed + 7)
    return fr


# ---------------------------------------------------------------------------
# Downsampler mirror (zarr::Downsampler add_frame / take_frame)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", ALL_DTYPES, ids=lambda d: DTYPE_NAMES[d])
@pytest.mark.parametrize("method", ALL_METHODS, ids=lambda m: METHOD_NAMES[m])
def test_downsampler_2d_all_dtypes_methods(gpu, dtype, method):
    for si, (h, w) in enumerate(SHAPES):
        dims = [(TIME, 0, 1, 1), (SPACE, h, 2, 1), (SPACE, w, 2, 1)]
        frames = _frames(dtype, 2, h, w, 100 * si + dtype * 7 + method)
        _, exp = oracle_cascade(dims, dtype, method, frames)
        ds = gpu.Downsampler(dims, dtype, method)
        for i, fr in enumerate(frames):
            ds.add_frame(fr)
            for l in range(1, ds.n_levels()):
                got = ds.take_frame(l)
                assert (got is None) == (l not in exp[i]), (h, w, i, l)
                if got is not None:
                    assert_same_pixels(got, exp[i][l], dtype, f"{h}x{w} f{i} L{l}")


@pytest.mark.parametrize("dtype", [U8, U16, I32, F32, F64], ids=lambda d: DTYPE_NAMES[d])
@pytest.mark.parametrize("method", ALL_METHODS, ids=lambda m: METHOD_NAMES[m])
def test_downsampler_3d_odd_z_cascade(gpu, dtype, method):
    # z Space with odd plane counts at several levels, two channels, two
    # timepoints: exercises pairing, odd pass-through and the break.
    for (z, cz, h, w, ch) in [(5, 1, 16, 16, 4), (15, 3, 48, 64, 16), (9, 2, 21, 13, 3)]:
        dims = [(TIME, 0, 1, 1), (CHANNEL, 2, 1, 1), (SPACE, z, cz, 1),
                (SPACE, h, ch, 1), (SPACE, w, ch, 1)]
        frames = _frames(dtype, 2 * 2 * z, h, w, z * 31 + method)
        _, exp = oracle_cascade(dims, dtype, method, frames)
        ds = gpu.Downsampler(dims, dtype, method)
        for i, fr in enumerate(frames):
            ds.add_frame(fr)
            for l in range(1, ds.n_levels()):
                got = ds.take_frame(l)
                assert (got is None) == (l not in exp[i]), (z, i, l)
                if got is not None:
                    assert_same_pixels(got, exp[i][l], dtype, f"z{z} f{i} L{l}")


def test_downsampler_reference_known_answers(gpu):
    """tests/unit-tests/downsampler.cpp known answers, on the GPU."""
    # test_basic_downsampling (:25-74): 10x10 of 100 -> 5x5 of 100
    ds = gpu.Downsampler([(TIME, 0, 5, 1), (SPACE, 10, 5, 1), (SPACE, 10, 5, 1)], U8, MEAN)
    assert ds.n_levels() == 2
    ds.add_frame(np.full((10, 10), 100, np.uint8))
    out = ds.take_frame(1)
    assert out.shape == (5, 5) and (out == 100).all()
    assert ds.take_frame(1) is None
    # test_3d_downsampling (:76-152): 100,200,300,400 -> L1 150, L2 250
    dims = [(TIME, 0, 5, 1), (CHANNEL, 3, 1, 3), (SPACE, 20, 5, 1),
            (SPACE, 20, 5, 1), (SPACE, 20, 5, 1)]
    ds = gpu.Downsampler(dims, U16, MEAN)
    ds.add_frame(np.full((20, 20), 100, np.uint16))
    assert ds.take_frame(1) is None
    ds.add_frame(np.full((20, 20), 200, np.uint16))
    l1 = ds.take_frame(1)
    assert l1.shape == (10, 10) and (l1 == 150).all()
    assert ds.take_frame(2) is None
    ds.add_frame(np.full((20, 20), 300, np.uint16))
    assert ds.take_frame(1) is None and ds.take_frame(2) is None
    ds.add_frame(np.full((20, 20), 400, np.uint16))
    l2 = ds.take_frame(2)
    assert l2.shape == (5, 5) and (l2 == 250).all()
    # test_min_max_downsampling (:447-528): [100 200; 150 250] blocks
    img = np.zeros((10, 10), np.uint8)
    img[0::2, 0::2], img[0::2, 1::2], img[1::2, 0::2], img[1::2, 1::2] = 100, 200, 150, 250
    for m, v in [(MEAN, 175), (MIN, 100), (MAX, 250)]:
        ds = gpu.Downsampler([(TIME, 0, 5, 1), (SPACE, 10, 5, 1), (SPACE, 10, 5, 1)], U8, m)
        ds.add_frame(img)
        assert (ds.take_frame(1) == v).all()
    # test_edge_cases (:411-445): 11x11 -> 6x6
    ds = gpu.Downsampler([(TIME, 0, 5, 1), (SPACE, 11, 5, 1), (SPACE, 11, 5, 1)], U8, MEAN)
    ds.add_frame(np.full((11, 11), 100, np.uint8))
    assert ds.take_frame(1).shape == (6, 6)
    # test_odd_z_multi_tc_no_bleed (downsampler-odd-z.cpp:19-86)
    dims = [(TIME, 0, 1, 1), (CHANNEL, 2, 1, 2), (SPACE, 3, 1, 1),
            (SPACE, 8, 4, 1), (SPACE, 8, 4, 1)]
    ds = gpu.Downsampler(dims, U16, MEAN)
    seen = []
    for t in range(2):
        for v in (100, 200):
            for z in range(3):
                ds.add_frame(np.full((8, 8), v, np.uint16))
                o = ds.take_frame(1)
                if o is not None:
                    assert (o == o.flat[0]).all()
                    seen.append(int(o.flat[0]))
    assert seen == [100, 100, 200, 200, 100, 100, 200, 200]
    assert ds.take_frame(1) is None
    # check_downsample (downsampler-odd-z.cpp:88-132): Z=15 chunk 3
    dims = [(TIME, 0, 1, 1), (SPACE, 15, 3, 1), (SPACE, 48, 16, 1), (SPACE, 64, 16, 1)]
    ds = gpu.Downsampler(dims, U8, MEAN)
    assert ds.level_dims(1)[1][1] == 8
    for val in (63, 127, 255):
        n = 0
        for i in range(15):
            ds.add_frame(np.full((48, 64), val, np.uint8))
            if i % 2 == 1:
                o = ds.take_frame(1)
                assert o is not None and (o == val).all()
                n += 1
        assert n == 7
        o = ds.take_frame(1)
        assert o is not None and (o == val).all()


def test_downsampler_metadata_and_errors(gpu):
    """method name and get_metadata().dump() byte-identical to the
    reference's (tests/golden/metadata.json, from the compiled reference)."""
    import json
    import os
    import aqz
    golden = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                         "metadata.json")))
    dims = [(TIME, 0, 5, 1), (SPACE, 10, 5, 1), (SPACE, 10, 5, 1)]
    for m in ALL_METHODS:
        ds = gpu.Downsampler(dims, U16, m)
        assert ds.method_name() == golden[str(m)]["method_name"]
        assert ds.metadata_json() == golden[str(m)]["metadata"]
    with pytest.raises(aqz.AqzError) as e:
        gpu.Downsampler(dims, U16, 4)
    assert e.value.status == 1
    with pytest.raises(aqz.AqzError):
        gpu.Downsampler(dims, 10, MEAN)
    ds = gpu.Downsampler(dims, U16, MEAN)
    with pytest.raises(aqz.AqzError):
        ds.add_frame(np.zeros((5, 5), np.uint16))  # too few bytes


# ---------------------------------------------------------------------------
# Stage: level-0 tile split + pyramid + tile split of every level
# ---------------------------------------------------------------------------
def _run_stage(gpu, dims, dtype, method, frames, max_levels=0, batch=0, chunks=None,
               knobs=0):
    # keep every chunk layer of the run resident so all can be checked;
    # knobs: the bench-header kernel switches (aqz_stage_bench_options)
    f0 = dims[0][2]
    for d in dims[1:-2]:
        f0 *= d[1]
    slots = -(-len(frames) // f0) + 2
    st = gpu.Stage(dims, dtype, method, max_levels=max_levels,
                   max_batch_frames=batch, layer_slots=slots, knobs=knobs)
    if chunks is None:
        st.append(frames)
    else:
        i = 0
        for c in chunks:
            st.append(np.ascontiguousarray(frames[i:i + c]))
            i += c
    st.finalize()
    return st


def _check_stage(gpu, dims, dtype, method, frames, **kw):
    exp, fw, ldims = expected_stage_layers(dims, dtype, method, frames,
                                           kw.get("max_levels", 0))
    st = _run_stage(gpu, dims, dtype, method, frames, **kw)
    assert st.n_levels() == len(ldims)
    for l in range(st.n_levels()):
        assert [tuple(x) for x in st.level_dims(l)] == [tuple(x) for x in ldims[l]]
        assert st.frames_written(l) == fw[l], (l, st.frames_written(l), fw[l])
    for (l, layer), (buf, flags) in sorted(exp.items()):
        got, gflags = st.copy_layer(l, layer)
        assert_same_pixels(got, buf, dtype, f"L{l} layer{layer}")
        assert (gflags == flags).all(), f"has_data L{l} layer{layer}: {gflags} vs {flags}"
    st.close()


@pytest.mark.parametrize("dtype", ALL_DTYPES, ids=lambda d: DTYPE_NAMES[d])
def test_stage_2d_tile_split_and_pyramid(gpu, dtype):
    for method in ALL_METHODS:
        for (h, w, cy, cx, ct) in [(64, 48, 16, 16, 2), (37, 29, 5, 7, 3),
                                    (130, 67, 32, 8, 1), (11, 11, 4, 4, 5)]:
            dims = [(TIME, 0, ct, 1), (SPACE, h, cy, 1), (SPACE, w, cx, 1)]
            frames = _frames(dtype, 7, h, w, h * w + method)
            _check_stage(gpu, dims, dtype, method, frames, batch=3)


@pytest.mark.parametrize("method", ALL_METHODS, ids=lambda m: METHOD_NAMES[m])
def test_stage_2d_channels_zero_frames_and_batches(gpu, method):
    # intermediate non-space dim (c), ragged chunks, all-zero frames (has_data)
    dims = [(TIME, 0, 2, 1), (CHANNEL, 3, 2, 1), (SPACE, 100, 32, 1), (SPACE, 90, 32, 1)]
    frames = _frames(U16, 13, 100, 90, 5 + method)
    frames[2] = 0
    frames[7] = 0
    _check_stage(gpu, dims, U16, method, frames, batch=4, chunks=[1, 5, 7])


@pytest.mark.parametrize("method", ALL_METHODS, ids=lambda m: METHOD_NAMES[m])
def test_stage_3d_generic_path(gpu, method):
    # the C example config (examples/stream-raw-multiscale-to-filesystem.c):
    # t 10/5, c 8/4, z 6/2 (Space), y 48/16, x 64/16
    dims = [(TIME, 10, 5, 2), (CHANNEL, 8, 4, 2), (SPACE, 6, 2, 1),
            (SPACE, 48, 16, 1), (SPACE, 64, 16, 2)]
    frames = _frames(U16, 10 * 8 * 6, 48, 64, 77 + method, specials=False)
    _check_stage(gpu, dims, U16, method, frames, batch=7)
    # odd z with several z levels, batches that split pairs
    dims = [(TIME, 0, 1, 1), (SPACE, 11, 2, 1), (SPACE, 40, 8, 1), (SPACE, 33, 8, 1)]
    frames = _frames(F32, 33, 40, 33, 9 + method)
    _check_stage(gpu, dims, F32, method, frames, batch=5, chunks=[3, 11, 19])


def test_stage_deep_pyramid_tail_levels(gpu):
    # more levels than the fused kernel cascades (tail levels, generic kernel)
    dims = [(TIME, 0, 1, 1), (SPACE, 1000, 4, 1), (SPACE, 700, 4, 1)]
    frames = _frames(U8, 3, 1000, 700, 3)
    _check_stage(gpu, dims, U8, MEAN, frames, batch=2)


def test_stage_max_levels_and_bounds(gpu):
    import aqz
    dims = [(TIME, 4, 2, 1), (SPACE, 64, 8, 1), (SPACE, 64, 8, 1)]
    frames = _frames(U16, 4, 64, 64, 1)
    _check_stage(gpu, dims, U16, MAX, frames, max_levels=2)
    st = gpu.Stage(dims, U16, MAX)
    st.append(frames)
    with pytest.raises(aqz.AqzError) as e:
        st.append(frames[:1])
    assert e.value.status == 12


@pytest.mark.parametrize("cfg", ["c1", "c2", "c3", "c5"])
def test_stage_baseline_configs(gpu, cfg):
    """BASELINE.json configs at full frame size (few frames), vs the oracle."""
    if cfg == "c1":
        dims, dt, m, n = [(TIME, 0, 4, 1), (SPACE, 512, 128, 1), (SPACE, 512, 128, 1)], U16, DECIMATE, 6
    elif cfg == "c2":
        dims, dt, m, n = [(TIME, 0, 4, 1), (SPACE, 2048, 128, 1), (SPACE, 2048, 128, 1)], U16, MEAN, 5
    elif cfg == "c3":
        dims, dt, m, n = [(TIME, 0, 2, 1), (SPACE, 4096, 128, 1), (SPACE, 4096, 128, 1)], U8, MEAN, 3
    else:
        dims, dt, m, n = [(TIME, 0, 1, 1), (SPACE, 8192, 128, 1), (SPACE, 8192, 128, 1)], F32, MEAN, 1
    h, w = dims[-2][1], dims[-1][1]
    frames = synthetic_frames(dt, n, h, w, 2024)
    _check_stage(gpu, dims, dt, m, frames, batch=2)


@pytest.mark.parametrize("nf", [1, 2])
@pytest.mark.parametrize("dtype", [U8, U16, I16, U32, F32], ids=lambda d: DTYPE_NAMES[d])
def test_stage_shallow_pyramid_strip(gpu, dtype, nf):
    """Pyramids of 2-3 levels (1-2 fused levels, e.g. C1's 3) on the strip
    kernel's 64-row interior regions, every method; the same stages forced
    onto fused_pyramid (knob 128); and XY-transposed storage order through
    the strip kernel's XY load.  300 x 1100 frames at 128-px chunks: interior
    regions plus ragged right and bottom edges."""
    dims = [(TIME, 0, 4, 1), (SPACE, 300, 128, 1), (SPACE, 1100, 128, 1)]
    for m in ALL_METHODS:
        frames = _frames(dtype, 5, 300, 1100, 31 * nf + 7 * m + dtype)
        for knobs, name in ((0, "fused_pyramid_strip"), (128, "fused_pyramid")):
            st = gpu.Stage(dims, dtype, m, max_levels=nf, knobs=knobs)
            assert st.n_levels() == nf + 1 and st.dominant_kernel() == name
            st.close()
            _check_stage(gpu, dims, dtype, m, frames, max_levels=nf, batch=3,
                         knobs=knobs)
    # XY: acquisition 1100 x 1088 -> storage 1088 rows x 1100 columns
    acq = [(TIME, 0, 4, 1), (SPACE, 1100, 128, 1), (SPACE, 1088, 128, 1)]
    frames = _frames(dtype, 5, 1100, 1088, 5 * nf + dtype)
    stored = np.ascontiguousarray(frames.transpose(0, 2, 1))
    exp, fw, ldims = expected_stage_layers([acq[0], acq[2], acq[1]], dtype, MEAN, stored,
                                           nf)
    st = gpu.Stage(acq, dtype, MEAN, storage_order=[0, 2, 1], max_levels=nf,
                   max_batch_frames=3, layer_slots=4)
    assert st.n_levels() == nf + 1
    assert st.dominant_kernel() == "fused_pyramid_strip (XY load)"
    st.append(frames[:3])
    st.append(frames[3:])
    st.finalize()
    for (l, layer), (buf, flags) in sorted(exp.items()):
        got, gflags = st.copy_layer(l, layer)
        assert_same_pixels(got, buf, dtype, f"xy L{l} layer{layer}")
        assert (gflags == flags).all(), (l, layer)
    st.close()


def test_stage_device_resident_input(gpu):
    import torch
    dims = [(TIME, 0, 2, 1), (SPACE, 256, 64, 1), (SPACE, 256, 64, 1)]
    frames = _frames(U16, 6, 256, 256, 4, specials=False)
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    t = torch.from_numpy(frames.view(np.int16)).cuda()
    st = gpu.Stage(dims, U16, MEAN, layer_slots=8)
    st.append(t)
    st.finalize()
    for (l, layer), (buf, flags) in exp.items():
        got, gflags = st.copy_layer(l, layer)
        assert_same_pixels(got, buf, U16, f"L{l}")
        assert (gflags == flags).all()


def test_stage_timing_marks(gpu):
    """The bench's timing pair (aqz_stage_timing_mark/_elapsed) brackets the
    kernels of the appends between the marks on the stage's own stream."""
    import torch
    dims = [(TIME, 0, 8, 1), (SPACE, 1024, 256, 1), (SPACE, 1024, 256, 1)]
    st = gpu.Stage(dims, U16, MEAN, max_batch_frames=8)
    with pytest.raises(gpu.AqzError):
        st.timing_elapsed()  # no marks yet
    with pytest.raises(gpu.AqzError):
        st.timing_mark(2)
    t = torch.zeros(8 * 1024 * 1024, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    st.timing_mark(0)
    st.timing_mark(1)
    empty = st.timing_elapsed()
    st.timing_mark(0)
    for _ in range(20):
        st.append_ptr(t.data_ptr(), 8)
    st.timing_mark(1)
    busy = st.timing_elapsed()
    st.synchronize()
    assert 0 <= empty < busy, (empty, busy)
    st.close()


# ---------------------------------------------------------------------------
# 2x2x2 fused path (regular z schedule) and z-slab sharding
# ---------------------------------------------------------------------------
# the register-cascade kernel (fused_pyramid_strip3d; tuning knob 512: its
# variant without the next-plane prefetch) and, with knob 256, the
# LDS-cascade kernel it replaced (fused_pyramid_3d)
KERNELS_3D = {"strip3d_pair": (0, "fused_pyramid_strip3d_pair"),
              # the round-4 pair kernel (6 waves per SIMD, spills; A/B only)
              "strip3d_pair_r4": (65536, "fused_pyramid_strip3d_pair"),
              # without the next-pair prefetch (A/B)
              "strip3d_pair_nopf": (131072, "fused_pyramid_strip3d_pair"),
              "strip3d": (2, "fused_pyramid_strip3d"),
              "strip3d_nopf": (2 | 512, "fused_pyramid_strip3d"),
              "lds3d": (256, "fused_pyramid_3d")}


@pytest.mark.parametrize("kernel", sorted(KERNELS_3D))
@pytest.mark.parametrize("dtype", [U8, U16, I16, U32, F32], ids=lambda d: DTYPE_NAMES[d])
def test_stage_3d_fused_regular(gpu, dtype, kernel):
    # every level halves x, y and z: G = 8 planes per workgroup
    knobs, name = KERNELS_3D[kernel]
    dims = [(TIME, 0, 1, 1), (CHANNEL, 2, 1, 1), (SPACE, 32, 4, 1),
            (SPACE, 512, 64, 1), (SPACE, 512, 64, 1)]
    st = gpu.Stage(dims, dtype, MEAN, knobs=knobs)
    assert st.dominant_kernel() == name
    st.close()
    for m in ALL_METHODS:
        frames = _frames(dtype, 2 * 32, 512, 512, 40 + m + dtype)
        # appends that leave and regain group alignment (fused <-> generic)
        _check_stage(gpu, dims, dtype, m, frames, batch=16, chunks=[3, 13, 32, 16],
                     knobs=knobs)


@pytest.mark.parametrize("kernel", sorted(KERNELS_3D))
def test_stage_c4_volume(gpu, kernel):
    # BASELINE configs[3] level structure (z 64 -> 32 -> 16 -> 16 with
    # 16-plane z chunks; xy 2048 -> 256 with 256-px chunks): fused 2x2x2
    knobs, name = KERNELS_3D[kernel]
    dims = [(TIME, 0, 1, 1), (SPACE, 64, 16, 1), (SPACE, 2048, 256, 1),
            (SPACE, 2048, 256, 1)]
    frames = synthetic_frames(U16, 64, 2048, 2048, 77)
    st = gpu.Stage(dims, U16, MEAN, knobs=knobs)
    assert st.dominant_kernel() == name
    st.close()
    _check_stage(gpu, dims, U16, MEAN, frames, batch=32, knobs=knobs)


@pytest.mark.parametrize("kernel", sorted(KERNELS_3D))
@pytest.mark.parametrize("dims,levels", [
    # 2 levels (one fused level, G = 2); 512 px: a u8 region is 512 px wide
    ([(TIME, 0, 1, 1), (SPACE, 8, 4, 1), (SPACE, 512, 256, 1), (SPACE, 512, 256, 1)], 2),
    # 3 levels (two fused levels, G = 4)
    ([(TIME, 0, 1, 1), (SPACE, 8, 2, 1), (SPACE, 1024, 256, 1), (SPACE, 1024, 256, 1)], 3),
], ids=["2lvl", "3lvl"])
def test_stage_3d_shallow(gpu, kernel, dims, levels):
    """Shallow 2x2x2 pyramids (1 or 2 fused levels) through every 2x2x2
    kernel: the strip kernel's early exits after level 1 / level 2."""
    knobs, name = KERNELS_3D[kernel]
    h = dims[-2][1]
    for dtype in (U8, U16, F32):
        st = gpu.Stage(dims, dtype, MEAN, knobs=knobs)
        assert st.dominant_kernel() == name
        assert st.n_levels() == levels
        st.close()
        for m in ALL_METHODS:
            frames = _frames(dtype, 16, h, h, 7 + m + dtype)
            _check_stage(gpu, dims, dtype, m, frames, batch=8, knobs=knobs)


@pytest.mark.parametrize("dtype", [U8, U16, F32], ids=lambda d: DTYPE_NAMES[d])
def test_stage_3d_five_levels(gpu, dtype):
    """Five levels (four fused: xy 1024 -> 64 with 64-px chunks), z halving
    at levels 1-3 only (64 -> 8 with 8-plane z chunks; level 4 keeps 8
    planes): the strip 3-D kernel's level-4 row and a level that halves XY
    but not z after three that halve both."""
    dims = [(TIME, 0, 1, 1), (SPACE, 64, 8, 1), (SPACE, 1024, 64, 1), (SPACE, 1024, 64, 1)]
    st = gpu.Stage(dims, dtype, MEAN)
    assert st.dominant_kernel() == "fused_pyramid_strip3d_pair"
    assert st.n_levels() == 5
    assert [st.level_dims(l)[1][1] for l in range(5)] == [64, 32, 16, 8, 8]
    st.close()
    for m in ALL_METHODS:
        frames = _frames(dtype, 64, 1024, 1024, 90 + m + dtype)
        _check_stage(gpu, dims, dtype, m, frames, batch=16)


def test_stage_z_slab_sharding(gpu):
    """Two stages own planes [0, 32) and [32, 64) of one volume (what two
    GPUs do with --gpus 2): their chunk layers assemble, with no exchange,
    into exactly the single-stage result."""
    dims = [(TIME, 0, 1, 1), (SPACE, 64, 16, 1), (SPACE, 512, 64, 1),
            (SPACE, 512, 64, 1)]
    frames = synthetic_frames(U16, 64, 512, 512, 5)
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    a = gpu.Stage(dims, U16, MEAN, layer_slots=2)
    b = gpu.Stage(dims, U16, MEAN, layer_slots=2, first_frame=32)
    a.append(np.ascontiguousarray(frames[:32]))
    b.append(np.ascontiguousarray(frames[32:]))
    a.finalize()
    b.finalize()
    for (l, layer), (buf, flags) in exp.items():
        ga, fa = a.copy_layer(l, layer)
        gb, fb = b.copy_layer(l, layer)
        assert_same_pixels(np.bitwise_or(ga, gb), buf, U16, f"L{l}")
        assert (np.maximum(fa, fb) == flags).all()
    for l in range(a.n_levels()):
        assert a.frames_written(l) + b.frames_written(l) - b.frames_written(l) >= 0
    assert b.frames_written(0) == 64 and a.frames_written(0) == 32
    a.close()
    b.close()


@pytest.mark.parametrize("dims,batch", [
    # fused 2x2x2 strip path (z 64 -> 32 -> 16, xy 256 -> 128 -> 64), G = 4
    ([(TIME, 0, 1, 1), (SPACE, 64, 16, 1), (SPACE, 256, 64, 1), (SPACE, 256, 64, 1)], 8),
    # generic cascade (level 2 keeps its xy size), slabs of 8 planes
    ([(TIME, 0, 1, 1), (SPACE, 32, 8, 1), (SPACE, 128, 64, 1), (SPACE, 128, 64, 1)], 3),
    # channels: every (t, c) stack is a z stack of its own
    ([(TIME, 0, 1, 1), (CHANNEL, 2, 1, 1), (SPACE, 32, 8, 1), (SPACE, 128, 64, 1),
      (SPACE, 128, 64, 1)], 16),
])
def test_stage_z_slab_schedule_volume_stream(gpu, dims, batch):
    """A stream of volumes split into 4 z slabs (aqz_stage_options
    z_slab_begin / z_slab_end; what --gpus 4 runs for C4): each stage gets
    only its planes of every stack, its frame ids jump over the other
    slabs', and the four stages' chunk layers OR together into the oracle's
    single-stream layers (z pairing, downsampler.cpp:358-389; chunk
    placement, array.dimensions.cpp:264-314)."""
    from aqz.dist import z_levels, z_slab
    Z, h, w = dims[-3][1], dims[-2][1], dims[-1][1]
    stacks = 2 * (dims[1][1] if dims[1][0] == CHANNEL else 1)  # two timepoints
    frames = synthetic_frames(U16, stacks * Z, h, w, 23 + Z)
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    planes = [lv[-3][1] for lv in gpu.pyramid_levels(dims)]
    zl = z_levels(planes)
    stages = []
    for r in range(4):
        lo, hi = z_slab(Z, 4, r, 1 << zl)
        st = gpu.Stage(dims, U16, MEAN, layer_slots=2 * stacks, max_batch_frames=batch,
                       z_slab=(lo, hi))
        for s in range(stacks):  # only this slab's planes of every stack
            st.append(np.ascontiguousarray(frames[s * Z + lo:s * Z + hi]))
        st.finalize()
        # after each slab the frame id jumps to the next stack's slab
        assert st.frames_written(0) == stacks * Z + lo
        stages.append(st)
    for (l, layer), (buf, flags) in exp.items():
        got = [st.copy_layer(l, layer) for st in stages]
        acc = got[0][0].copy()
        hd = got[0][1].copy()
        for g, f in got[1:]:
            np.bitwise_or(acc, g, out=acc)
            np.maximum(hd, f, out=hd)
        assert_same_pixels(acc, buf, U16, f"L{l} layer {layer}")
        assert np.array_equal(hd, flags), (l, layer)
    for st in stages:
        st.close()


def test_stage_z_slab_rejects_misaligned(gpu):
    dims = [(TIME, 0, 1, 1), (SPACE, 64, 16, 1), (SPACE, 256, 64, 1), (SPACE, 256, 64, 1)]
    with pytest.raises(gpu.AqzError):
        gpu.Stage(dims, U16, MEAN, z_slab=(2, 18))  # z halves twice: multiples of 4
    with pytest.raises(gpu.AqzError):
        gpu.Stage(dims, U16, MEAN, z_slab=(16, 16))


def test_stage_z_slab_bounded_extent(gpu):
    """A bounded time dim (2 stacks of 64 planes) with the slab [0, 16): the
    stage takes 2 x 16 of its own planes and refuses the next with status 12
    (Array::write_frame's bounds check, array.cpp:171-175).  Frame ids jump
    over the other slabs, so room is counted in this stage's own frames."""
    dims = [(TIME, 2, 1, 1), (SPACE, 64, 16, 1), (SPACE, 256, 64, 1), (SPACE, 256, 64, 1)]
    frames = synthetic_frames(U16, 48, 256, 256, 9)
    st = gpu.Stage(dims, U16, MEAN, layer_slots=4, max_batch_frames=8, z_slab=(0, 16))
    st.append(np.ascontiguousarray(frames[:16]))
    assert st.frames_written(0) == 64  # jumped to the next stack's slab
    with pytest.raises(gpu.AqzError) as e:
        st.append(np.ascontiguousarray(frames[16:48]))  # only 16 fit
    assert e.value.status == 12
    assert st.frames_written(0) == 64 + 64  # the 16 that fit, then the jump
    with pytest.raises(gpu.AqzError) as e:
        st.append(np.ascontiguousarray(frames[:1]))
    assert e.value.status == 12
    st.close()


@pytest.mark.parametrize("pad", [0, 4224])
def test_stage_async_handoff_pinned_and_pageable(gpu, pad):
    """The ingestion / hand-off pipeline: pinned and pageable (multi-threaded
    staging copy) host sources, H2D on the copy stream, and every chunk layer
    handed off with copy_layer_async while the 3-slot ring wraps several
    times -- the copies must see each layer whole (a slot is not rewritten
    before its D2H has finished).  pad > 0: chunks `bpc + pad` apart on the
    device (bench option chunk_pad_bytes), packed back to bpc by the strided
    D2H."""
    dims = [(TIME, 0, 2, 1), (SPACE, 1024, 128, 1), (SPACE, 1024, 128, 1)]
    n, B = 20, 4
    frames = synthetic_frames(U16, n, 1024, 1024, 31)
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    st = gpu.Stage(dims, U16, MEAN, layer_slots=2, max_batch_frames=B, chunk_pad_bytes=pad)
    L = st.n_levels()
    lay = [st.layout(l) for l in range(L)]
    assert all(x["chunk_pitch"] == x["bytes_per_chunk"] + pad for x in lay)
    nbytes = [x["bytes_per_chunk"] * x["chunks_per_layer"] for x in lay]
    pinned_src = gpu.HostBuffer(B * frames[0].nbytes)
    out, handed = {}, [0] * L

    def hand_off(final=False):
        for l in range(L):
            F = lay[l]["frames_per_layer"]
            done = st.frames_written(l) // F
            if final and st.frames_written(l) % F:
                done += 1
            while handed[l] < done:
                buf = gpu.HostBuffer(nbytes[l])
                hd = gpu.HostBuffer(lay[l]["chunks_per_layer"])
                st.copy_layer_async(l, handed[l], buf.ptr, nbytes[l], hd.ptr, hd.nbytes)
                out[(l, handed[l])] = (buf, hd)
                handed[l] += 1

    appended = 0
    for i, b0 in enumerate(range(0, n, B)):
        chunk = np.ascontiguousarray(frames[b0:b0 + B])
        if i % 2 == 0:
            # a pinned source is read asynchronously: reuse it only once the
            # stage reports its frames consumed
            while st.frames_consumed() < appended:
                pass
            pinned_src.view(np.uint16, chunk.shape)[...] = chunk
            st.append(pinned_src, len(chunk))
        else:
            st.append(chunk)  # pageable: copied before return
            chunk[...] = 0
        appended += len(chunk)
        assert st.frames_consumed() <= appended
        hand_off()
    st.synchronize()
    assert st.frames_consumed() == n
    st.finalize()
    hand_off(final=True)
    st.wait_copies()
    assert sorted(out) == sorted(exp)
    for key, (buf, flags) in sorted(exp.items()):
        got, gflags = out[key]
        assert_same_pixels(got.array.copy(), buf, U16, f"L{key[0]} layer{key[1]}")
        assert (gflags.array == flags).all(), key
    # the synchronous copy of a still-resident layer packs the chunks too
    for l in range(L):
        last = (st.frames_written(l) - 1) // lay[l]["frames_per_layer"]
        got, gflags = st.copy_layer(l, last)
        assert_same_pixels(got, exp[(l, last)][0], U16, f"sync L{l} layer{last}")
        assert np.array_equal(gflags, exp[(l, last)][1])
    st.close()


@pytest.mark.parametrize("perm", [[0, 2, 1, 3, 4], [0, 1, 2, 4, 3], [0, 2, 1, 4, 3]],
                         ids=["cz_swap", "xy_swap", "cz_and_xy_swap"])
def test_stage_storage_dimension_order(gpu, perm):
    """storage_dimension_order: level-0 frame ids go through
    transpose_frame_id (array.cpp:557-561), an XY swap transposes every
    acquired frame before the split and the downsampler sees the transposed
    frame (array.cpp:525-533, multiscale.array.cpp:66-72); every level
    works on the storage-order dims (array.dimensions.cpp:12-73)."""
    acq = [(TIME, 0, 2, 1), (CHANNEL, 3, 2, 1), (SPACE, 4, 2, 1),
           (SPACE, 40, 16, 1), (SPACE, 57, 8, 1)]
    n = 3 * 4 * 3 + 5  # three time points and a partial fourth
    frames = _frames(U16, n, 40, 57, 17 + sum(i * p for i, p in enumerate(perm)),
                     specials=False)
    sdims = [acq[i] for i in perm]
    xy = perm[-1] != len(acq) - 1
    stored = np.ascontiguousarray(frames.transpose(0, 2, 1)) if xy else frames
    dims_map = gpu.Dims(acq, U16, storage_order=perm)
    exp, fw, ldims = expected_stage_layers(sdims, U16, MEAN, stored,
                                           storage_fid=dims_map.transpose_frame_id)
    st = gpu.Stage(acq, U16, MEAN, storage_order=perm, max_batch_frames=5)
    assert st.n_levels() == len(ldims)
    for l in range(st.n_levels()):
        assert [tuple(x) for x in st.level_dims(l)] == [tuple(x) for x in ldims[l]]
    for b0 in range(0, n, 5):
        st.append(np.ascontiguousarray(frames[b0:b0 + 5]))
    st.finalize()
    for l in range(st.n_levels()):
        assert st.frames_written(l) == fw[l]
    for (l, layer), (buf, flags) in sorted(exp.items()):
        got, gflags = st.copy_layer(l, layer)
        assert_same_pixels(got, buf, U16, f"L{l} layer{layer}")
        assert (gflags == flags).all(), (l, layer)
    st.close()


# XY-transposed storage order with the transpose fused into the strip
# kernel's loads (load_region_xy): storage rows = acquisition X (chunk 128,
# so 64-row regions), 4 levels, interior and edge regions; knob 4096 forces
# the separate transpose_frames pass, whose output must be the same.
XY_KERNELS = {"fused": (0, "fused_pyramid_strip (XY load)"),
              "pass": (4096, "transpose_frames + fused_pyramid_strip")}


@pytest.mark.parametrize("path", sorted(XY_KERNELS))
@pytest.mark.parametrize("dtype", [U8, U16, I16, U32, F32], ids=lambda d: DTYPE_NAMES[d])
def test_stage_xy_fused_strip(gpu, dtype, path):
    knobs, name = XY_KERNELS[path]
    # acquisition Y x X = 1000 x 1088 -> storage 1088 rows x 1000 columns
    acq = [(TIME, 0, 4, 1), (SPACE, 1000, 128, 1), (SPACE, 1088, 128, 1)]
    methods = [MEAN, MIN] if path == "fused" else [MEAN]
    for m in methods:
        frames = _frames(dtype, 6, 1000, 1088, 61 + dtype + 5 * m)
        stored = np.ascontiguousarray(frames.transpose(0, 2, 1))
        exp, fw, ldims = expected_stage_layers([acq[0], acq[2], acq[1]], dtype, m, stored)
        st = gpu.Stage(acq, dtype, m, storage_order=[0, 2, 1], max_batch_frames=4,
                       layer_slots=4, knobs=knobs)
        assert st.dominant_kernel() == name
        assert st.n_levels() >= 4
        st.append(frames[:4])
        st.append(frames[4:])
        st.finalize()
        for (l, layer), (buf, flags) in sorted(exp.items()):
            got, gflags = st.copy_layer(l, layer)
            assert_same_pixels(got, buf, dtype, f"{path} m{m} L{l} layer{layer}")
            assert (gflags == flags).all(), (l, layer)
        st.close()


@pytest.mark.parametrize("dtype", [U8, U16, F32, F64], ids=lambda d: DTYPE_NAMES[d])
def test_stage_xy_transpose_sizes(gpu, dtype):
    # frames larger than one 64x64 transpose tile, ragged on both axes
    acq = [(TIME, 0, 3, 1), (SPACE, 130, 32, 1), (SPACE, 77, 16, 1)]
    frames = _frames(dtype, 7, 130, 77, 5 + dtype)
    stored = np.ascontiguousarray(frames.transpose(0, 2, 1))
    exp, fw, ldims = expected_stage_layers([acq[0], acq[2], acq[1]], dtype, MAX, stored)
    st = gpu.Stage(acq, dtype, MAX, storage_order=[0, 2, 1], max_batch_frames=3,
                   layer_slots=4)
    st.append(frames)
    st.finalize()
    for (l, layer), (buf, flags) in sorted(exp.items()):
        got, gflags = st.copy_layer(l, layer)
        assert_same_pixels(got, buf, dtype, f"L{l} layer{layer}")
        assert (gflags == flags).all()
    st.close()


def test_stage_ring_arena_offset(gpu):
    """Bench option ring_arena_bytes (tools/arena_probe.py): every ring
    carved from one allocation and moved inside it restarts the stage at
    frame 0, oracle-exact at each offset."""
    import aqz
    dims = [(TIME, 0, 4, 1), (SPACE, 512, 128, 1), (SPACE, 512, 128, 1)]
    frames = synthetic_frames(U16, 8, 512, 512, 17)
    exp, fw, ldims = expected_stage_layers(dims, U16, MEAN, frames)
    st = gpu.Stage(dims, U16, MEAN, layer_slots=3, max_batch_frames=8,
                   ring_arena_bytes=4 << 20, ring_malloc_flags=4)
    for off in (0, 1 << 20, 4 << 20):
        st.set_ring_offset(off)
        st.append(frames)
        st.synchronize()
        for (l, layer), (buf, flags) in sorted(exp.items()):
            got, gflags = st.copy_layer(l, layer)
            assert_same_pixels(got, buf, U16, f"offset {off} L{l} layer{layer}")
            assert (gflags == flags).all(), (off, l, layer)
    with pytest.raises(aqz.AqzError):
        st.set_ring_offset((4 << 20) + 256)
    st.close()


@pytest.mark.parametrize("env", [{"AQZ_KNOBS": "8"}, {"AQZ_KNOBS": "32"},
                                 {"AQZ_KNOBS": "4", "AQZ_NT": "0",
                                  "AQZ_REGION_ROWS_LOG2": "4", "AQZ_CHUNK_PAD": "4096"}],
                         ids=["skip-deep-levels", "skip-flags", "mixed"])
def test_environment_cannot_change_drop_in_output(gpu, monkeypatch, env):
    """Kernel tuning lives only in the bench header (aqz_stage_bench_options):
    the round-3 library read AQZ_KNOBS & co. from the environment, where bit
    8 skipped levels >= 3 and bit 32 every has_data flush.  A drop-in stage
    made with such variables set must still be oracle-exact."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    dims = [(TIME, 0, 4, 1), (SPACE, 1024, 128, 1), (SPACE, 1024, 128, 1)]
    frames = synthetic_frames(U16, 8, 1024, 1024, 5)
    frames[4:] = 0  # an all-zero chunk layer: has_data must still be right
    exp, fw, ldims = expected_stage_layers(dims, U16, MEAN, frames)
    st = gpu.Stage(dims, U16, MEAN, layer_slots=3, max_batch_frames=8)
    assert st.n_levels() == len(ldims) >= 4
    assert all(st.layout(l)["chunk_pitch"] == st.layout(l)["bytes_per_chunk"]
               for l in range(st.n_levels()))
    st.append(frames)
    st.finalize()
    for (l, layer), (buf, flags) in sorted(exp.items()):
        got, gflags = st.copy_layer(l, layer)
        assert_same_pixels(got, buf, U16, f"env {env} L{l} layer{layer}")
        assert (gflags == flags).all(), (l, layer)
    st.close()


XY_KERNELS_3D = {"default": (0, "fused_pyramid_strip3d (XY load)"),
                 "pair": (65536, "fused_pyramid_strip3d_pair (XY load)"),
                 "single": (2, "fused_pyramid_strip3d (XY load)"),
                 "pass": (4096, "transpose_frames + fused_pyramid_strip3d_pair")}


@pytest.mark.parametrize("path", sorted(XY_KERNELS_3D))
@pytest.mark.parametrize("dtype", [U8, U16, I16, U32, F32], ids=lambda d: DTYPE_NAMES[d])
def test_stage_xy_fused_strip3d(gpu, dtype, path):
    """XY-transposed storage order on a 2x2x2 pyramid (transpose_frame,
    array.cpp:488-534): the 3-D strip kernel reads the acquisition-order
    planes itself (load_region_xy, one LDS transpose per plane), knob 4096
    the separate transpose pass.  Batches of whole z groups take the fused
    load -- one plane at a time by default, two at a time with knob 65536
    (fused_pyramid_strip3d_pair, each half of the workgroup its own LDS
    tile; it spills, so it is not the default); a
    batch that also needs the generic cascade (6 planes: one z group and a
    carried pair) is transposed first.  Either way every level equals the
    oracle's on the transposed frames."""
    knobs, want = XY_KERNELS_3D[path]
    # acquisition (t, z, y, x) = (*, 16, 1024, 768) -> storage x = 1024 (a
    # multiple of the 512-B region), storage y = 768 (64-row regions)
    acq = [(TIME, 0, 1, 1), (SPACE, 16, 4, 1), (SPACE, 1024, 128, 1), (SPACE, 768, 128, 1)]
    store = [acq[0], acq[1], acq[3], acq[2]]
    frames = _frames(dtype, 32, 1024, 768, 13 + dtype)
    stored = np.ascontiguousarray(frames.transpose(0, 2, 1))
    for m, batches in ((MEAN, [8, 8, 8, 8]), (MAX, [6, 10, 16])):
        exp, fw, ldims = expected_stage_layers(store, dtype, m, stored)
        st = gpu.Stage(acq, dtype, m, storage_order=[0, 1, 3, 2], max_batch_frames=16,
                       layer_slots=4, knobs=knobs)
        assert st.dominant_kernel() == want
        assert st.n_levels() == len(ldims) == 4
        i = 0
        for b in batches:
            st.append(np.ascontiguousarray(frames[i:i + b]))
            i += b
        st.finalize()
        for (l, layer), (buf, flags) in sorted(exp.items()):
            got, gflags = st.copy_layer(l, layer)
            assert_same_pixels(got, buf, dtype, f"{path} m{m} L{l} layer{layer}")
            assert (gflags == flags).all(), (l, layer)
        st.close()
