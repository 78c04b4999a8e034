"""CPU suite, part 1: the oracle is pinned before anything is checked
against it.

  * against the golden fixtures generated from the compiled reference
    (tests/golden/make_golden.py);
  * against the reference's own unit-test known answers
    (tests/unit-tests/downsampler*.cpp, array-dimensions-*.cpp), restated;
  * live against the compiled reference (oracle/_ref) on random cases, where
    it was built (this container).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_bindings as ob
from helpers import assert_same_pixels, with_specials

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _cascade_keys(z):
    return sorted({k.split("/")[0] for k in z.files})


def test_oracle_matches_golden_cascades():
    z = np.load(os.path.join(GOLDEN, "cascade_small.npz"), allow_pickle=False)
    keys = _cascade_keys(z)
    assert len(keys) >= 200
    n_frames = 0
    for key in keys:
        dims = [tuple(int(v) for v in d) for d in z[f"{key}/dims"]]
        dt, m = (int(v) for v in z[f"{key}/meta"])
        frames = z[f"{key}/in"]
        ds = ob.OracleDownsampler(dims, dt, m)
        for i in range(frames.shape[0]):
            ds.add_frame(frames[i])
            for lvl in range(1, ds.n_levels()):
                got = ds.take_frame(lvl)
                name = f"{key}/out/{i}/{lvl}"
                assert (got is None) == (name not in z.files), name
                if got is not None:
                    assert_same_pixels(got, z[name], dt, name)
                    n_frames += 1
    assert n_frames > 500


def test_oracle_matches_golden_tile_split():
    z = np.load(os.path.join(GOLDEN, "tile_split.npz"), allow_pickle=False)
    for key in sorted({k.split("/")[0] for k in z.files}):
        dims = [tuple(int(v) for v in d) for d in z[f"{key}/dims"]]
        dt = int(z[f"{key}/dtype"][0])
        od = ob.OracleDims(dims, dt)
        layer, flags = od.new_layer()
        frames = z[f"{key}/in"]
        for fid in range(frames.shape[0]):
            od.write_frame_to_chunks(fid, frames[fid], layer, flags)
        assert np.array_equal(layer, z[f"{key}/layer"]), key
        assert np.array_equal(flags, z[f"{key}/has_data"]), key
        assert flags.min() == 1 or not flags.all()


@pytest.mark.parametrize("key", ["c1_u16_512_decimate", "c2_u16_2048_mean_c128",
                                 "c4_u16_2048x64z_mean"])
def test_oracle_matches_golden_digests(key):
    rec = json.load(open(os.path.join(GOLDEN, "digests.json")))[key]
    dims = [tuple(d) for d in rec["dims"]]
    ds = ob.OracleDownsampler(dims, rec["dtype"], rec["method"])
    assert [list(map(list, ds.level_dims(l))) for l in range(ds.n_levels())] == rec["levels"]
    h, w = dims[-2][1], dims[-1][1]
    got = []
    for i in range(rec["frames"]):
        ds.add_frame(ob.synthetic_frames(rec["dtype"], 1, h, w, rec["seed"] + i)[0])
        for lvl in range(1, ds.n_levels()):
            img = ds.take_frame(lvl)
            if img is not None:
                got.append([i, lvl, hashlib.sha256(img.tobytes()).hexdigest()])
    assert got == rec["out"]


# ---------------------------------------------------------------------------
# Reference unit-test known answers (restated)
# ---------------------------------------------------------------------------
def test_kat_basic_and_3d():
    # downsampler.cpp:25-74
    ds = ob.OracleDownsampler([(ob.TIME, 0, 5, 1), (ob.SPACE, 10, 5, 1), (ob.SPACE, 10, 5, 1)],
                              ob.U8, ob.MEAN)
    assert ds.n_levels() == 2
    ds.add_frame(np.full((10, 10), 100, np.uint8))
    assert (ds.take_frame(1) == 100).all() and ds.take_frame(1) is None
    # downsampler.cpp:76-152
    dims = [(ob.TIME, 0, 5, 1), (ob.CHANNEL, 3, 1, 3), (ob.SPACE, 20, 5, 1),
            (ob.SPACE, 20, 5, 1), (ob.SPACE, 20, 5, 1)]
    ds = ob.OracleDownsampler(dims, ob.U16, ob.MEAN)
    seq = []
    for v in (100, 200, 300, 400):
        ds.add_frame(np.full((20, 20), v, np.uint16))
        seq.append((ds.take_frame(1), ds.take_frame(2)))
    assert seq[0] == (None, None)
    assert (seq[1][0] == 150).all() and seq[1][1] is None
    assert seq[2] == (None, None)
    assert (seq[3][1] == 250).all() and seq[3][1].shape == (5, 5)


def test_kat_methods_patterns_and_edges():
    img = np.zeros((10, 10), np.uint8)
    img[0::2, 0::2], img[0::2, 1::2], img[1::2, 0::2], img[1::2, 1::2] = 100, 200, 150, 250
    dims = [(ob.TIME, 0, 5, 1), (ob.SPACE, 10, 5, 1), (ob.SPACE, 10, 5, 1)]
    for m, v in [(ob.MEAN, 175), (ob.MIN, 100), (ob.MAX, 250)]:  # :447-528
        ds = ob.OracleDownsampler(dims, ob.U8, m)
        ds.add_frame(img)
        assert (ds.take_frame(1) == v).all()
    # gradient pattern, expected_mean = (v1+v2+v3+v4)/4 in int (:626-729)
    y, x = np.mgrid[0:8, 0:8]
    g = (100 + x * 20 + y * 50).astype(np.uint16)
    v1, v2, v3, v4 = g[0::2, 0::2], g[0::2, 1::2], g[1::2, 0::2], g[1::2, 1::2]
    dims = [(ob.TIME, 0, 5, 1), (ob.SPACE, 8, 4, 1), (ob.SPACE, 8, 4, 1)]
    exp = {ob.MEAN: ((v1.astype(int) + v2 + v3 + v4) // 4).astype(np.uint16),
           ob.MIN: np.minimum(np.minimum(v1, v2), np.minimum(v3, v4)),
           ob.MAX: np.maximum(np.maximum(v1, v2), np.maximum(v3, v4))}
    for m, e in exp.items():
        ds = ob.OracleDownsampler(dims, ob.U16, m)
        ds.add_frame(g)
        assert np.array_equal(ds.take_frame(1), e)
    # 11x11 -> 6x6 (:411-445)
    ds = ob.OracleDownsampler([(ob.TIME, 0, 5, 1), (ob.SPACE, 11, 5, 1), (ob.SPACE, 11, 5, 1)],
                              ob.U8, ob.MEAN)
    ds.add_frame(np.full((11, 11), 100, np.uint8))
    assert ds.take_frame(1).shape == (6, 6)
    # SURVEY §8c probe: 3x3 u16 [0..8]
    img = np.arange(9, dtype=np.uint16).reshape(3, 3)
    for m, e in [(ob.MEAN, [[2, 3], [6, 8]]), (ob.MIN, [[0, 2], [6, 8]]),
                 (ob.MAX, [[4, 5], [7, 8]]), (ob.DECIMATE, [[0, 2], [6, 8]])]:
        assert ob.oracle_scale_image(img, ob.U16, m).tolist() == e
    # integer semantics: trunc toward zero, 32-bit wrap
    a = np.array([[-1, -2], [-3, -4]], np.int8)
    assert ob.oracle_scale_image(a, ob.I8, ob.MEAN).tolist() == [[-2]]
    b = np.full((2, 2), 4_000_000_000, np.uint32)
    assert ob.oracle_scale_image(b, ob.U32, ob.MEAN).tolist() == [[778774528]]


def test_kat_level_geometry():
    # test_writer_configurations (:256-322): 5 levels, max(chunk, size >> l)
    dims = [(ob.TIME, 100, 10, 1), (ob.CHANNEL, 3, 3, 1), (ob.SPACE, 128, 8, 1),
            (ob.SPACE, 512, 64, 1), (ob.SPACE, 512, 64, 1)]
    ds = ob.OracleDownsampler(dims, ob.U16, ob.MEAN)
    assert ds.n_levels() == 5
    for l in range(1, 5):
        d = ds.level_dims(l)
        assert d[0][1] == 100 and d[1][1] == 3
        for i in range(2, 5):
            assert d[i][1] == max(dims[i][2], dims[i][1] >> l)
    # test_anisotropic_writer_configurations (:324-409)
    dims = [(ob.TIME, 100, 10, 1), (ob.CHANNEL, 3, 3, 1), (ob.SPACE, 1000, 128, 1),
            (ob.SPACE, 2000, 512, 1), (ob.SPACE, 2000, 256, 1)]
    ds = ob.OracleDownsampler(dims, ob.U16, ob.MEAN)
    assert ds.n_levels() == 4
    exp = {1: (500, 1000, 1000), 2: (250, 500, 500), 3: (125, 500, 500)}
    for l, (z, y, x) in exp.items():
        d = ds.level_dims(l)
        assert (d[2][1], d[3][1], d[4][1]) == (z, y, x)
        assert (d[2][2], d[3][2], d[4][2]) == (128, 512, 256)
    # test_max_levels (:730-785)
    dims = [(ob.TIME, 100, 10, 1), (ob.SPACE, 512, 64, 1), (ob.SPACE, 512, 64, 1)]
    assert ob.OracleDownsampler(dims, ob.U16, ob.MEAN, 2).n_levels() == 3
    assert ob.OracleDownsampler(dims, ob.U16, ob.MEAN, 0).n_levels() > 3
    # C2 with 256-px chunks is 4 levels, 5 with 128-px chunks
    c2 = [(ob.TIME, 0, 1, 1), (ob.SPACE, 2048, 256, 1), (ob.SPACE, 2048, 256, 1)]
    assert ob.OracleDownsampler(c2, ob.U16, ob.MEAN).n_levels() == 4
    c2[1], c2[2] = (ob.SPACE, 2048, 128, 1), (ob.SPACE, 2048, 128, 1)
    assert ob.OracleDownsampler(c2, ob.U16, ob.MEAN).n_levels() == 5


def test_kat_odd_z():
    # downsampler-odd-z.cpp:88-132
    dims = [(ob.TIME, 0, 1, 1), (ob.SPACE, 15, 3, 1), (ob.SPACE, 48, 16, 1), (ob.SPACE, 64, 16, 1)]
    ds = ob.OracleDownsampler(dims, ob.U8, ob.MEAN)
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
        assert (ds.take_frame(1) == val).all()
    # issue #226 no bleed (:19-86)
    dims = [(ob.TIME, 0, 1, 1), (ob.CHANNEL, 2, 1, 2), (ob.SPACE, 3, 1, 1),
            (ob.SPACE, 8, 4, 1), (ob.SPACE, 8, 4, 1)]
    ds = ob.OracleDownsampler(dims, ob.U16, ob.MEAN)
    seen = []
    for t in range(2):
        for v in (100, 200):
            for z in range(3):
                ds.add_frame(np.full((8, 8), v, np.uint16))
                o = ds.take_frame(1)
                if o is not None:
                    seen.append(int(o.flat[0]))
    assert seen == [100, 100, 200, 200, 100, 100, 200, 200]
    # SURVEY §8a a7 emission table: T.C.Z = inf.2.5 at 16^2, chunk 4, z chunk 1
    dims = [(ob.TIME, 0, 1, 1), (ob.CHANNEL, 2, 1, 1), (ob.SPACE, 5, 1, 1),
            (ob.SPACE, 16, 4, 1), (ob.SPACE, 16, 4, 1)]
    ds = ob.OracleDownsampler(dims, ob.U16, ob.MEAN)
    assert [ds.level_dims(l)[2][1] for l in range(ds.n_levels())] == [5, 3, 2, 1]
    emitted = []
    for i in range(10):
        ds.add_frame(np.zeros((16, 16), np.uint16))
        emitted.append([l for l in range(1, 4) if ds.take_frame(l) is not None])
    assert emitted[:5] == [[], [1], [], [1, 2], [1, 2, 3]]


TILE_GROUP_OFFSET = [0, 0, 12, 12, 24, 0, 0, 12, 12, 24, 36, 36, 48, 48, 60]


def test_kat_index_tables():
    # array-dimensions-tile-group-offset.cpp / -chunk-internal-offset.cpp
    dims = [(ob.TIME, 0, 5, 0), (ob.CHANNEL, 3, 2, 0), (ob.SPACE, 5, 2, 0),
            (ob.SPACE, 48, 16, 0), (ob.SPACE, 64, 16, 0)]
    od = ob.OracleDims(dims, ob.F32)
    tgo = [od.tile_group_offset(i) for i in range(76)]
    assert tgo[:15] == TILE_GROUP_OFFSET and tgo[15:30] == TILE_GROUP_OFFSET
    assert tgo[75] == 0
    od16 = ob.OracleDims(dims, ob.U16)
    cio = [od16.chunk_internal_offset(i) for i in range(76)]
    assert cio[:15] == [0, 512, 0, 512, 0, 1024, 1536, 1024, 1536, 1024, 0, 512, 0, 512, 0]
    assert cio[15:20] == [2048, 2560, 2048, 2560, 2048]
    assert cio[60:66] == [8192, 8704, 8192, 8704, 8192, 9216] and cio[75] == 0


# ---------------------------------------------------------------------------
# Live against the compiled reference (this container only)
# ---------------------------------------------------------------------------
needs_ref = pytest.mark.skipif(not ob.ref_available(), reason="oracle/_ref not built")


@needs_ref
def test_oracle_vs_reference_random_cascades():
    rng = np.random.default_rng(7)
    for trial in range(120):
        dt = int(rng.integers(0, 10))
        m = int(rng.integers(0, 4))
        w, h = int(rng.integers(1, 60)), int(rng.integers(1, 60))
        cw, ch = int(rng.integers(1, 16)), int(rng.integers(1, 16))
        if rng.random() < 0.5:
            z, cz = int(rng.integers(1, 10)), int(rng.integers(1, 4))
            dims = [(ob.TIME, 0, 1, 1), (ob.CHANNEL, 2, 1, 1), (ob.SPACE, z, cz, 1),
                    (ob.SPACE, h, ch, 1), (ob.SPACE, w, cw, 1)]
            n = 4 * z
        else:
            dims = [(ob.TIME, 0, 1, 1), (ob.SPACE, h, ch, 1), (ob.SPACE, w, cw, 1)]
            n = 2
        ml = int(rng.integers(0, 3))
        frames = with_specials(ob.synthetic_frames(dt, n, h, w, trial), dt, trial)
        a = ob.OracleDownsampler(dims, dt, m, ml)
        b = ob.OracleDownsampler(dims, dt, m, ml, use_ref=True)
        assert a.n_levels() == b.n_levels()
        for l in range(a.n_levels()):
            assert a.level_dims(l) == b.level_dims(l)
        for i in range(n):
            a.add_frame(frames[i])
            b.add_frame(frames[i])
            for l in range(1, a.n_levels()):
                x, y = a.take_frame(l), b.take_frame(l)
                assert (x is None) == (y is None)
                if x is not None:
                    assert_same_pixels(x, y, dt, f"trial {trial} f{i} L{l}")


@needs_ref
def test_oracle_vs_reference_index_math_and_split():
    rng = np.random.default_rng(8)
    for trial in range(80):
        nd = int(rng.integers(3, 6))
        dims = [(ob.TIME, 0, int(rng.integers(1, 6)), 1)]
        for _ in range(nd - 3):
            dims.append((int(rng.integers(0, 3)), int(rng.integers(1, 7)),
                         int(rng.integers(1, 4)), 1))
        dims += [(ob.SPACE, int(rng.integers(1, 40)), int(rng.integers(1, 12)), 1),
                 (ob.SPACE, int(rng.integers(1, 40)), int(rng.integers(1, 12)), 1)]
        dt = int(rng.integers(0, 10))
        o, r = ob.OracleDims(dims, dt), ob.OracleDims(dims, dt, use_ref=True)
        for fid in range(40):
            assert o.tile_group_offset(fid) == r.tile_group_offset(fid)
            assert o.chunk_internal_offset(fid) == r.chunk_internal_offset(fid)
        la, ha = o.new_layer()
        lb, hb = r.new_layer()
        fr = ob.synthetic_frames(dt, 6, dims[-2][1], dims[-1][1], trial)
        fr[::3] = 0
        for fid in range(6):
            assert o.write_frame_to_chunks(fid, fr[fid], la, ha) == \
                r.write_frame_to_chunks(fid, fr[fid], lb, hb)
        assert np.array_equal(la, lb) and np.array_equal(ha, hb)
