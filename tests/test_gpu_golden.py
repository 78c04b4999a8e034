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
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle_bindings import NP_DTYPES, OracleDims, synthetic_frames

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DIGESTS = json.load(open(os.path.join(GOLDEN, "digests.json")))
BPP = {k: np.dtype(v).itemsize for k, v in NP_DTYPES.items()}


def _inputs(rec):
    h, w = rec["dims"][-2][1], rec["dims"][-1][1]
    return [synthetic_frames(rec["dtype"], 1, h, w, rec["seed"] + i)[0]
            for i in range(rec["frames"])]


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


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
                got.append([i, lvl, _sha(img)])
    assert got == rec["out"]


@pytest.mark.parametrize("key", sorted(DIGESTS))
def test_stage_matches_reference_digests(gpu, key):
    rec = DIGESTS[key]
    dims = [tuple(d) for d in rec["dims"]]
    dt = rec["dtype"]
    frames = np.stack(_inputs(rec))
    n = len(frames)
    st = gpu.Stage(dims, dt, rec["method"], max_batch_frames=n, layer_slots=2)
    assert st.n_levels() == len(rec["levels"])
    st.append(frames)
    st.finalize()
    # expected level-frame digests in emission order, per level
    want = {}
    for _, lvl, sha in rec["out"]:
        want.setdefault(lvl, []).append(sha)
    want[0] = [_sha(f) for f in frames]
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
            got.append(_sha(untile_frame(od, ldims, dt, layers[fid // F], fid % F)))
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
