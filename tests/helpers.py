"""Shared test helpers: bit-exact comparison and oracle-side expectations."""
from __future__ import annotations

import numpy as np

from oracle_bindings import (F32, F64, NP_DTYPES, OracleDims, OracleDownsampler)


def assert_same_pixels(got: np.ndarray, exp: np.ndarray, dtype: int, what: str = ""):
    """Bit-exact for integers.  Floats: bit-exact for every non-NaN value
    (+-0, denormals, +-inf included) and NaN exactly where the reference has
    NaN; the NaN payload/sign is not compared (the reference's own payload
    depends on the host compiler's operand order -- see DESIGN.md)."""
    npdt = NP_DTYPES[dtype]
    g = np.ascontiguousarray(got).view(npdt).reshape(-1)
    e = np.ascontiguousarray(exp).view(npdt).reshape(-1)
    assert g.shape == e.shape, f"{what}: shape {g.shape} != {e.shape}"
    if dtype in (F32, F64):
        gn, en = np.isnan(g), np.isnan(e)
        bad_nan = np.flatnonzero(gn != en)
        assert bad_nan.size == 0, f"{what}: NaN mismatch at {bad_nan[:8]}"
        ui = np.uint32 if dtype == F32 else np.uint64
        gb, eb = g.view(ui)[~gn], e.view(ui)[~en]
        bad = np.flatnonzero(gb != eb)
        assert bad.size == 0, (f"{what}: {bad.size} mismatches, first at "
                               f"{bad[:8]}: got {g[~gn][bad[:4]]} exp {e[~en][bad[:4]]}")
    else:
        bad = np.flatnonzero(g != e)
        assert bad.size == 0, (f"{what}: {bad.size} mismatches, first at {bad[:8]}: "
                               f"got {g[bad[:4]]} exp {e[bad[:4]]}")


def with_specials(frames: np.ndarray, dtype: int, seed: int, frac: float = 0.2):
    """Sprinkle edge values: dtype min/max for integers; NaN, +-0, +-inf,
    denormals and huge values for floats."""
    rng = np.random.default_rng(seed)
    f = frames.reshape(-1)
    npdt = NP_DTYPES[dtype]
    if dtype in (F32, F64):
        tiny = np.finfo(npdt).tiny
        sp = np.array([np.nan, -np.nan, 0.0, -0.0, np.inf, -np.inf, tiny / 4,
                       -tiny / 3, np.finfo(npdt).max, -np.finfo(npdt).max, 1.0],
                      dtype=npdt)
    else:
        ii = np.iinfo(npdt)
        sp = np.array([ii.min, ii.max, 0, 1, ii.max - 1], dtype=npdt)
    idx = rng.integers(0, f.size, size=max(1, int(f.size * frac)))
    f[idx] = sp[rng.integers(0, sp.size, size=idx.size)]
    return frames


def oracle_cascade(dims, dtype, method, frames, max_levels=0):
    """Per input frame, the dict {level: image} the reference's
    add_frame + take_frame sequence yields (C restatement)."""
    ds = OracleDownsampler(dims, dtype, method, max_levels)
    out = []
    for fr in frames:
        ds.add_frame(fr)
        got = {}
        for l in range(1, ds.n_levels()):
            img = ds.take_frame(l)
            if img is not None:
                got[l] = img
        out.append(got)
    return ds, out


def expected_stage_layers(dims, dtype, method, frames, max_levels=0,
                          level_dims=None, storage_fid=None):
    """Chunk layers {(level, layer): (bytes, has_data)} that
    MultiscaleArray::write_frame produces for `frames`
    (multiscale.array.cpp:57-74, 291-325): level 0 tile split, then every
    level's emitted frames tile-split in emission order.  `storage_fid`
    optionally maps a level-0 acquisition frame id to its storage id."""
    ds = OracleDownsampler(dims, dtype, method, max_levels)
    L = ds.n_levels()
    ldims = level_dims or [ds.level_dims(l) for l in range(L)]
    od = [OracleDims(ldims[l], dtype) for l in range(L)]
    layers = {}
    fw = [0] * L

    def put(level, img):
        fid = fw[level]
        fw[level] += 1
        F = od[level].frames_per_chunk_layer()
        key = (level, fid // F)
        if key not in layers:
            layers[key] = od[level].new_layer()
        sfid = storage_fid(fid) if (level == 0 and storage_fid) else fid
        od[level].write_frame_to_chunks(sfid, img, *layers[key])

    for fr in frames:
        put(0, fr)
        ds.add_frame(fr)
        for l in range(1, L):
            img = ds.take_frame(l)
            if img is not None:
                put(l, img)
    return layers, fw, ldims


def layer_pixels(buf: np.ndarray, dtype: int) -> np.ndarray:
    return buf.view(NP_DTYPES[dtype])


def assemble_layers(layers, dims, dtype) -> np.ndarray:
    """The stored array a zarr reader sees, from chunk layers {layer: bytes}
    of storage-order `dims` [(type, size, chunk, shard)]: the regular chunk
    grid in C order (zarr v3), chunk layer k = append indices
    [k*c0, (k+1)*c0), chunks of a layer in C order over dims 1..n-1, each
    chunk a C-order block of the chunk shape (ragged edges padded)."""
    npdt = NP_DTYPES[dtype]
    sizes = [d[1] for d in dims]
    chunks = [d[2] for d in dims]
    n_layers = max(layers) + 1
    if sizes[0] == 0:
        sizes[0] = n_layers * chunks[0]
    grid = [-(-s // c) for s, c in zip(sizes[1:], chunks[1:])]
    padded = [n_layers * chunks[0]] + [g * c for g, c in zip(grid, chunks[1:])]
    out = np.zeros(padded, dtype=npdt)
    per_chunk = int(np.prod(chunks))
    for k, buf in layers.items():
        px = np.frombuffer(bytes(buf), dtype=npdt)
        for ci, idx in enumerate(np.ndindex(*grid)):
            block = px[ci * per_chunk:(ci + 1) * per_chunk].reshape(chunks)
            sl = [slice(k * chunks[0], (k + 1) * chunks[0])]
            sl += [slice(j * c, (j + 1) * c) for j, c in zip(idx, chunks[1:])]
            out[tuple(sl)] = block
    return out[tuple(slice(0, s) for s in sizes)]
