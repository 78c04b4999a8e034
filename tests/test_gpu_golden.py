"""GPU output pinned directly to the REFERENCE's own outputs.

tests/golden/digests.json holds the sha256 of every level frame that the
compiled reference (oracle/_ref: downsampler.cpp, Downsampler::add_frame /
take_frame, downsampler.cpp:306-414) emitted for BASELINE-shaped inputs
regenerated from recorded splitmix64 seeds (tests/golden/make_golden.py).
Here the same inputs go through the HIP path and every level frame's
digest must equal the reference's:

* `aqz.Downsampler` (the frame-by-frame add/take surface);
* `aqz.Stage` (the batched stage): its chunk layers are un-tiled back into
  level frames by an inverse of Array::write_frame_to_chunks_
  (array.cpp:507-622) over the oracle's ArrayDimensions index math
  (tile_group_offset / chunk_internal_offset, array.dimensions.cpp:264-314,
  pinned to the reference on the CPU), then hashed.

tile_split.npz (the reference's chunk layers + has_data for ragged tile
geometries, Chunk::write_tile_rows chunk.cpp:17-67) is compared byte for
byte with the stage's level-0 layer.

cascade_small.npz (every level frame the compiled reference emitted for 10
dtypes x 4 methods x odd shapes, specials included, and odd-z 3-D cascades
with channels) is replayed through aqz.Downsampler and aqz.Stage and
compared frame by frame (NaN-equivalent for floats, tests/helpers.py).

The *_specials digest cases sprinkle dtype min/max (integers: the 8/16-bit
truncation toward zero and 32/64-bit wrap of mean4, downsampler.cpp:46-51)
and NaN / +-0 / +-inf / denormals (floats) into full-size frames; float
digests hash the frame with its NaNs canonicalised.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from helpers import assert_same_pixels, with_specials
from oracle_bindings import F32, F64, NP_DTYPES, OracleDims, synthetic_frames

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DIGESTS = json.load(open(os.path.join(GOLDEN, "digests.json")))
BPP = {k: np.dtype(v).itemsize for k, v in NP_DTYPES.items()}


def _inputs(rec):
    """The digest case's input frames (make_golden.py digest_frame)."""
    h, w = rec["dims"][-2][1], rec["dims"][-1][1]
    out = []
    for i in range(rec["frames"]):
        fr = synthetic_frames(rec["dtype"], 1, h, w, rec["seed"] + i)
        if rec.get("specials"):
            fr = with_specials(fr, rec["dtype"], rec["seed"] + i + 7919, frac=0.05)
        out.append(fr[0])
    return out


def _sha(a, dtype=None):
    """sha256 of a level frame; float NaNs canonicalised (make_golden.py
    frame_digest)."""
    a = np.ascontiguousarray(a)
    if dtype in (F32, F64):
        a = a.view(NP_DTYPES[dtype]).copy()
        a[np.isnan(a)] = np.nan
    return hashlib.sha256(a.tobytes()).hexdigest()


def untile_frame(od, dims, dtype, layer, fid):
    """Level frame `fid` (storage frame id) out of its chunk layer: the
    inverse of write_frame_to_chunks_ (array.cpp:537-619)."""
    bpp = BPP[dtype]
    H, th = dims[-2][1], dims[-2][2]
    W, tw = dims[-1][1], dims[-1][2]
    ntx = -(-W // tw)
    bpc = od.bytes_per_chunk()
    grp = od.tile_group_offset(fid)
    inner = od.chunk_internal_offset(fid)
    out = np.empty((H, W * bpp), dtype=np.uint8)
    for ty in range(-(-H // th)):
        for tx in range(ntx):
            c = ty * ntx + tx + grp
            rows = min(th, H - ty * th)
            cols = min(tw, W - tx * tw) * bpp
            base = c * bpc + inner
            blk = layer[base:base + th * tw * bpp].reshape(th, tw * bpp)
            out[ty * th:ty * th + rows, tx * tw * bpp:tx * tw * bpp + cols] = \
                blk[:rows, :cols]
    return out.view(NP_DTYPES[dtype])


@pytest.mark.parametrize("key", sorted(DIGESTS))
def test_downsampler_matches_reference_digests(gpu, key):
    rec = DIGESTS[key]
    ds = gpu.Downsampler([tuple(d) for d in rec["dims"]], rec["dtype"], rec["method"])
    assert ds.n_levels() == len(rec["levels"])
    for lvl, ld in enumerate(rec["levels"]):
        assert [tuple(x) for x in ds.level_dims(lvl)] == [tuple(x) for x in ld], lvl
    got = []
    for i, fr in enumerate(_inputs(rec)):
        ds.add_frame(fr)
        for lvl in range(1, ds.n_levels()):
            img = ds.take_frame(lvl)
            if img is not None:
                got.append([i, lvl, _sha(img, rec["dtype"])])
    assert got == rec["out"]


@pytest.mark.parametrize("key", sorted(DIGESTS))
def test_stage_matches_reference_digests(gpu, key):
    rec = DIGESTS[key]
    dims = [tuple(d) for d in rec["dims"]]
    dt = rec["dtype"]
    frames = np.stack(_inputs(rec))
    n = len(frames)
    if n >= 128:
        # a whole volume stream: irregular appends (a few planes, then runs
        # that start mid z group), every layer kept resident for the check
        parts, B, slots = [3, 61, 64, 128], 128, 8
    else:
        parts, B, slots = [n], n, 2
    assert sum(parts) == n
    st = gpu.Stage(dims, dt, rec["method"], max_batch_frames=B, layer_slots=slots)
    assert st.n_levels() == len(rec["levels"])
    i = 0
    for p in parts:
        st.append(np.ascontiguousarray(frames[i:i + p]))
        i += p
    st.finalize()
    # expected level-frame digests in emission order, per level
    want = {}
    for _, lvl, sha in rec["out"]:
        want.setdefault(lvl, []).append(sha)
    want[0] = [_sha(f, dt) for f in frames]
    for lvl in range(st.n_levels()):
        ldims = [tuple(x) for x in rec["levels"][lvl]]
        assert [tuple(x) for x in st.level_dims(lvl)] == ldims, lvl
        od = OracleDims(ldims, dt)
        F = od.frames_per_chunk_layer()
        nf = st.frames_written(lvl)
        assert nf == len(want.get(lvl, [])), (lvl, nf)
        layers = {}
        got = []
        for fid in range(nf):
            if fid // F not in layers:
                layers[fid // F] = st.copy_layer(lvl, fid // F)[0]
            got.append(_sha(untile_frame(od, ldims, dt, layers[fid // F], fid % F), dt))
        assert got == want.get(lvl, []), f"{key} level {lvl}"
    st.close()


def _tile_cases():
    z = np.load(os.path.join(GOLDEN, "tile_split.npz"), allow_pickle=False)
    keys = sorted({k.split("/")[0] for k in z.files})
    return z, keys


def test_stage_tile_split_matches_reference_layers(gpu):
    z, keys = _tile_cases()
    for key in keys:
        dims = [tuple(int(v) for v in d) for d in z[f"{key}/dims"]]
        dt = int(z[f"{key}/dtype"][0])
        frames = z[f"{key}/in"]
        st = gpu.Stage(dims, dt, 0, multiscale=False, max_batch_frames=len(frames))
        st.append(np.ascontiguousarray(frames))
        st.finalize()
        layer, flags = st.copy_layer(0, 0)
        assert np.array_equal(layer, z[f"{key}/layer"]), key
        assert np.array_equal(flags, z[f"{key}/has_data"]), key
        st.close()


def _cascade_cases():
    z = np.load(os.path.join(GOLDEN, "cascade_small.npz"), allow_pickle=False)
    keys = sorted({k.split("/")[0] for k in z.files})
    return z, keys


CASCADE, CASCADE_KEYS = _cascade_cases()


def _cascade(key):
    z = CASCADE
    dims = [tuple(int(v) for v in d) for d in z[f"{key}/dims"]]
    dt, m = (int(v) for v in z[f"{key}/meta"])
    frames = z[f"{key}/in"]
    out = {}
    for k in z.files:
        if k.startswith(f"{key}/out/"):
            i, lvl = (int(v) for v in k.split("/")[2:4])
            out[(i, lvl)] = z[k]
    return dims, dt, m, frames, out


@pytest.mark.parametrize("group", ["2d", "3d"])
def test_downsampler_replays_reference_cascades(gpu, group):
    """Every frame of tests/golden/cascade_small.npz (the compiled
    reference's add_frame / take_frame outputs) through aqz.Downsampler:
    the same frames at the same steps and levels, bit-exact (floats
    NaN-equivalent)."""
    keys = [k for k in CASCADE_KEYS if k.startswith(group)]
    assert keys
    for key in keys:
        dims, dt, m, frames, out = _cascade(key)
        ds = gpu.Downsampler(dims, dt, m)
        matched = 0
        for i, fr in enumerate(frames):
            ds.add_frame(np.ascontiguousarray(fr))
            for lvl in range(1, ds.n_levels()):
                img = ds.take_frame(lvl)
                exp = out.get((i, lvl))
                assert (img is None) == (exp is None), (key, i, lvl)
                if exp is not None:
                    assert_same_pixels(img, exp, dt, f"{key} frame {i} L{lvl}")
                    matched += 1
        assert matched == len(out), key


@pytest.mark.parametrize("group", ["2d", "3d"])
def test_stage_replays_reference_cascades(gpu, group):
    """The same fixtures through aqz.Stage (appended in two irregular
    batches): every level's frames, un-tiled from its chunk layers in
    emission order, equal the reference's."""
    keys = [k for k in CASCADE_KEYS if k.startswith(group)]
    for key in keys:
        dims, dt, m, frames, out = _cascade(key)
        n = len(frames)
        st = gpu.Stage(dims, dt, m, max_batch_frames=max(1, n), layer_slots=n + 2)
        cut = n // 3
        for a, b in ((0, cut), (cut, n)):
            if b > a:
                st.append(np.ascontiguousarray(frames[a:b]))
        st.finalize()
        for lvl in range(st.n_levels()):
            ldims = [tuple(x) for x in st.level_dims(lvl)]
            exp = [frames[i] for i in range(n)] if lvl == 0 else \
                [out[(i, l)] for (i, l) in sorted(out) if l == lvl]
            assert st.frames_written(lvl) == len(exp), (key, lvl)
            od = OracleDims(ldims, dt)
            F = od.frames_per_chunk_layer()
            layers = {}
            for fid, e in enumerate(exp):
                if fid // F not in layers:
                    layers[fid // F] = st.copy_layer(lvl, fid // F)[0]
                img = untile_frame(od, ldims, dt, layers[fid // F], fid % F)
                assert_same_pixels(img, e, dt, f"{key} L{lvl} frame {fid}")
        st.close()
