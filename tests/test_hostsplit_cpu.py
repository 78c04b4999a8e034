"""The level-0 tile split on the host (aqz_dims_split_frame_rows; the stage's
aqz_stage_split_level0_host / _rows run the same code over the stage's
level-0 ArrayDimensions), against the reference's own loop: the compiled
ArrayDimensions + Chunk::write_tile_rows driving array.cpp:537-619
(oracle/_ref, ref_write_frame_to_chunks), and the C restatement where the
reference is not built.  CPU only: the split is host code."""
import numpy as np
import pytest

import aqz
import oracle_bindings as ob

BPP = {ob.U8: 1, ob.U16: 2, 2: 4, 3: 8, ob.F32: 4}


def _frames(dt, n, h, w, seed):
    return ob.synthetic_frames(dt, n, h, w, seed)


def _random_dims(rng):
    nd = int(rng.integers(3, 6))
    dims = [(ob.TIME, int(rng.integers(0, 3)) * 4, int(rng.integers(1, 5)),
             int(rng.integers(1, 3)))]
    for _ in range(nd - 3):
        dims.append((int(rng.integers(0, 3)), int(rng.integers(1, 6)),
                     int(rng.integers(1, 4)), 1))
    dims += [(ob.SPACE, int(rng.integers(1, 70)), int(rng.integers(1, 17)), 1),
             (ob.SPACE, int(rng.integers(1, 70)), int(rng.integers(1, 17)), 1)]
    return dims


def _split_layer(a, frames, fids, rng, chunk0=0, n_chunks=None):
    """Split `frames` (ids fids) with aqz over random row ranges, as several
    threads would."""
    bpc = a.bytes_per_chunk()
    n = n_chunks if n_chunks is not None else a.number_of_chunks_in_memory() - chunk0
    layer = np.zeros(bpc * n, dtype=np.uint8)
    has = np.zeros(n, dtype=np.uint8)
    for f, fid in zip(frames, fids):
        H = f.shape[0]
        cuts = sorted(set([0, H] + [int(x) for x in rng.integers(0, H + 1, size=3)]))
        for r0, r1 in zip(cuts[:-1], cuts[1:]):
            a.split_frame_rows(f, fid, layer, has, r0, r1, chunk0=chunk0)
    return layer, has


def test_host_split_matches_the_oracle_restatement():
    rng = np.random.default_rng(61)
    for case in range(120):
        dims = _random_dims(rng)
        dt = [ob.U8, ob.U16, ob.F32, 3][case % 4]
        a, o = aqz.Dims(dims, dt), ob.OracleDims(dims, dt)
        F = a.frames_per_chunk_layer()
        H, W = dims[-2][1], dims[-1][1]
        first = int(rng.integers(0, 3)) * F
        n = int(min(F, 12))
        fr = _frames(dt, n, H, W, 1000 + case)
        if case % 5 == 0:
            fr[1:3] = 0  # frames without data
        fids = list(range(first, first + n))
        layer, has = _split_layer(a, fr, fids, rng)
        ol, oh = o.new_layer()
        for f, fid in zip(fr, fids):
            o.write_frame_to_chunks(fid, f, ol, oh)
        assert np.array_equal(layer, ol), (case, dims, dt)
        assert np.array_equal(has, oh), (case, dims, dt)


@pytest.mark.skipif(not ob.ref_available(), reason="oracle/_ref not built")
def test_host_split_matches_the_compiled_reference_with_storage_orders():
    """The reference transposes the acquisition frame id to storage order
    (array.cpp:557-561) before the lattice math; the split does the same."""
    rng = np.random.default_rng(62)
    for case in range(60):
        inner = [(ob.CHANNEL, int(rng.integers(1, 4)), 1, 1),
                 (ob.SPACE, int(rng.integers(1, 6)), int(rng.integers(1, 3)), 1),
                 (ob.OTHER, int(rng.integers(1, 3)), 1, 1)]
        H, W = int(rng.integers(3, 40)), int(rng.integers(3, 40))
        dims = [(ob.TIME, 0, int(rng.integers(1, 3)), 1)] + inner + \
               [(ob.SPACE, H, int(rng.integers(2, 12)), 1),
                (ob.SPACE, W, int(rng.integers(2, 12)), 1)]
        perm = [0] + [1 + int(i) for i in rng.permutation(3)] + [4, 5]
        dt = [ob.U16, ob.U8, ob.F32][case % 3]
        a = aqz.Dims(dims, dt, storage_order=perm)
        r = ob.OracleDims(dims, dt, use_ref=True, order=perm)
        F = a.frames_per_chunk_layer()
        fr = _frames(dt, F, H, W, 2000 + case)
        layer, has = _split_layer(a, fr, range(F), rng)
        rl, rh = r.new_layer()
        for fid in range(F):
            r.write_frame_to_chunks(r.transpose_frame_id(fid), fr[fid], rl, rh)
        assert np.array_equal(layer, rl), (case, dims, perm)
        assert np.array_equal(has, rh), (case, dims, perm)


def test_host_split_into_dim1_bands():
    """A dim-1 band (chunk0 = band * chunks_per_band) receives exactly the
    band's slice of the layer (Array::flush_completed_bands_,
    array.cpp:873-908)."""
    rng = np.random.default_rng(63)
    dims = [(ob.TIME, 0, 1, 1), (ob.SPACE, 10, 4, 1), (ob.SPACE, 36, 16, 1),
            (ob.SPACE, 40, 16, 1)]
    a, o = aqz.Dims(dims, ob.U16), ob.OracleDims(dims, ob.U16)
    ok, n_bands, fpb, cpb = a.dim1_banding()
    assert ok and n_bands == 3 and fpb == 4
    F = a.frames_per_chunk_layer()
    fr = _frames(ob.U16, F, 36, 40, 7)
    ol, oh = o.new_layer()
    for fid in range(F):
        o.write_frame_to_chunks(fid, fr[fid], ol, oh)
    bpc = a.bytes_per_chunk()
    for b in range(n_bands):
        lo, hi = b * fpb, min((b + 1) * fpb, F)
        layer, has = _split_layer(a, fr[lo:hi], range(lo, hi), rng, chunk0=b * cpb,
                                  n_chunks=cpb)
        assert np.array_equal(layer, ol[b * cpb * bpc:(b + 1) * cpb * bpc])
        assert np.array_equal(has, oh[b * cpb:(b + 1) * cpb])
    # a frame of band 1 does not fit band 0's chunks
    layer = np.zeros(bpc * cpb, dtype=np.uint8)
    has = np.zeros(cpb, dtype=np.uint8)
    with pytest.raises(aqz.AqzError) as e:
        a.split_frame_rows(fr[fpb], fpb, layer, has)
    assert e.value.status == 1


def test_host_split_bc2_geometry_and_refusals():
    """C2's level 0 (2048^2 u16, 256^2 chunks, t-chunk 64): whole frames;
    an XY-transposed storage order is refused (status 9)."""
    dims = [(ob.TIME, 0, 64, 1), (ob.SPACE, 2048, 256, 8), (ob.SPACE, 2048, 256, 8)]
    a, o = aqz.Dims(dims, ob.U16), ob.OracleDims(dims, ob.U16)
    fr = _frames(ob.U16, 3, 2048, 2048, 5)
    bpc = a.bytes_per_chunk()
    layer = np.zeros(bpc * 64, dtype=np.uint8)
    has = np.zeros(64, dtype=np.uint8)
    ol, oh = o.new_layer()
    for fid in (0, 1, 63):
        f = fr[fid % 3]
        a.split_frame_rows(f, fid, layer, has)
        o.write_frame_to_chunks(fid, f, ol, oh)
    assert np.array_equal(layer, ol) and np.array_equal(has, oh)
    # short destination / has_data
    with pytest.raises(aqz.AqzError):
        a.split_frame_rows(fr[0], 0, layer[:bpc * 10], has)
    xy = aqz.Dims(dims, ob.U16, storage_order=[0, 2, 1])
    with pytest.raises(aqz.AqzError) as e:
        xy.split_frame_rows(fr[0], 0, layer, has)
    assert e.value.status == 9
