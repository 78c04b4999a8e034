#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the COMPILED REFERENCE
(oracle/_ref/libaqzref.so = /root/reference/src/streaming/{downsampler,
array.dimensions,zarr.common,chunk}.cpp built by oracle/Makefile).

Run here (where /root/reference exists):  python tests/golden/make_golden.py
Outputs (data only -- inputs and expected outputs):
  cascade_small.npz   raw inputs + every emitted level frame, small shapes,
                      10 dtypes x 4 methods, 2-D and 3-D (odd z) cascades
  tile_split.npz      ragged tile-split layers + has_data flags
  digests.json        sha256 of every level frame for BASELINE-sized configs
                      (inputs regenerated from splitmix64 seeds)
  metadata.json       Downsampler::downsampling_method() and
                      get_metadata().dump() per method (downsampler.cpp:
                      422-485): the OME block MultiscaleArray embeds in
                      zarr.json (`make_golden.py metadata` writes only this)
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_bindings as ob  # noqa: E402
from helpers import with_specials  # noqa: E402

SHAPES_2D = [(2, 2), (3, 3), (5, 7), (11, 11), (37, 29)]
CASES_3D = [(5, 1, 16, 16, 4), (9, 2, 21, 13, 3)]  # z, cz, h, w, chunk


def cascade_cases():
    """(key, dims, dtype, method, frames) for the small cascade fixtures."""
    out = []
    for dt in range(10):
        for m in range(4):
            for si, (h, w) in enumerate(SHAPES_2D):
                dims = [(ob.TIME, 0, 1, 1), (ob.SPACE, h, 2, 1), (ob.SPACE, w, 2, 1)]
                seed = 1000 * dt + 100 * m + si
                fr = with_specials(ob.synthetic_frames(dt, 1, h, w, seed), dt, seed + 1)
                out.append((f"2d_{ob.DTYPE_NAMES[dt]}_{ob.METHOD_NAMES[m]}_{h}x{w}",
                            dims, dt, m, fr))
            if dt in (ob.U8, ob.U16, ob.I16, ob.F32):
                for ci, (z, cz, h, w, ch) in enumerate(CASES_3D):
                    dims = [(ob.TIME, 0, 1, 1), (ob.CHANNEL, 2, 1, 1), (ob.SPACE, z, cz, 1),
                            (ob.SPACE, h, ch, 1), (ob.SPACE, w, ch, 1)]
                    seed = 5000 + 1000 * dt + 100 * m + ci
                    fr = with_specials(ob.synthetic_frames(dt, 2 * 2 * z, h, w, seed), dt,
                                       seed + 1)
                    out.append((f"3d_{ob.DTYPE_NAMES[dt]}_{ob.METHOD_NAMES[m]}_z{z}",
                                dims, dt, m, fr))
    return out


TILE_CASES = [
    # (key, dims, dtype) -- ragged x/y tiles, ragged intermediate dims
    ("even_u16", [(ob.TIME, 0, 2, 1), (ob.CHANNEL, 3, 2, 1), (ob.SPACE, 5, 2, 1),
                  (ob.SPACE, 48, 16, 1), (ob.SPACE, 64, 16, 1)], ob.U16),
    ("ragged_xy_f32", [(ob.TIME, 0, 2, 1), (ob.SPACE, 37, 8, 1), (ob.SPACE, 29, 7, 1)], ob.F32),
    ("ragged_all_u8", [(ob.TIME, 0, 3, 1), (ob.CHANNEL, 5, 2, 1), (ob.SPACE, 19, 6, 1),
                       (ob.SPACE, 23, 5, 1)], ob.U8),
]

# BASELINE.json configs (frame sizes as named; few frames) + the 3-D one at
# a reduced plane count with the same level structure.
DIGEST_CASES = [
    ("c1_u16_512_decimate", [(ob.TIME, 0, 4, 1), (ob.SPACE, 512, 128, 1), (ob.SPACE, 512, 128, 1)],
     ob.U16, ob.DECIMATE, 4),
    ("c2_u16_2048_mean_c128", [(ob.TIME, 0, 4, 1), (ob.SPACE, 2048, 128, 1), (ob.SPACE, 2048, 128, 1)],
     ob.U16, ob.MEAN, 3),
    ("c3_u8_4096_mean", [(ob.TIME, 0, 2, 1), (ob.SPACE, 4096, 128, 1), (ob.SPACE, 4096, 128, 1)],
     ob.U8, ob.MEAN, 2),
    ("c4_u16_2048x64z_mean", [(ob.TIME, 0, 1, 1), (ob.SPACE, 64, 16, 1), (ob.SPACE, 2048, 256, 1),
                              (ob.SPACE, 2048, 256, 1)], ob.U16, ob.MEAN, 64),
    ("c5_f32_8192_mean", [(ob.TIME, 0, 1, 1), (ob.SPACE, 8192, 128, 1), (ob.SPACE, 8192, 128, 1)],
     ob.F32, ob.MEAN, 1),
    # round 4: the other methods, the signed / wrapping integer types and
    # float specials at full frame sizes, and C4 at BASELINE's geometry
    ("c2_u16_2048_min_c128", [(ob.TIME, 0, 4, 1), (ob.SPACE, 2048, 128, 1),
                              (ob.SPACE, 2048, 128, 1)], ob.U16, ob.MIN, 2),
    ("c2_u16_2048_max_c128", [(ob.TIME, 0, 4, 1), (ob.SPACE, 2048, 128, 1),
                              (ob.SPACE, 2048, 128, 1)], ob.U16, ob.MAX, 2),
    ("i8_1000x1030_mean_specials", [(ob.TIME, 0, 2, 1), (ob.SPACE, 1000, 64, 1),
                                    (ob.SPACE, 1030, 64, 1)], ob.I8, ob.MEAN, 2),
    ("i16_1024_mean_specials", [(ob.TIME, 0, 2, 1), (ob.SPACE, 1024, 128, 1),
                                (ob.SPACE, 1024, 128, 1)], ob.I16, ob.MEAN, 2),
    ("i32_1024_mean_specials", [(ob.TIME, 0, 2, 1), (ob.SPACE, 1024, 128, 1),
                                (ob.SPACE, 1024, 128, 1)], ob.I32, ob.MEAN, 2),
    ("u32_777x1001_max_specials", [(ob.TIME, 0, 2, 1), (ob.SPACE, 777, 64, 1),
                                   (ob.SPACE, 1001, 64, 1)], ob.U32, ob.MAX, 2),
    ("u64_512_mean_specials", [(ob.TIME, 0, 2, 1), (ob.SPACE, 512, 64, 1),
                               (ob.SPACE, 512, 64, 1)], ob.U64, ob.MEAN, 2),
    ("i64_300x700_min_specials", [(ob.TIME, 0, 2, 1), (ob.SPACE, 300, 32, 1),
                                  (ob.SPACE, 700, 32, 1)], ob.I64, ob.MIN, 2),
    ("f32_2048_mean_specials", [(ob.TIME, 0, 2, 1), (ob.SPACE, 2048, 128, 1),
                                (ob.SPACE, 2048, 128, 1)], ob.F32, ob.MEAN, 2),
    ("f32_1536_min_specials", [(ob.TIME, 0, 2, 1), (ob.SPACE, 1536, 128, 1),
                               (ob.SPACE, 1536, 128, 1)], ob.F32, ob.MIN, 2),
    ("f64_512_max_specials", [(ob.TIME, 0, 2, 1), (ob.SPACE, 512, 64, 1),
                              (ob.SPACE, 512, 64, 1)], ob.F64, ob.MAX, 2),
    ("f64_600x500_decimate_specials", [(ob.TIME, 0, 2, 1), (ob.SPACE, 600, 64, 1),
                                       (ob.SPACE, 500, 64, 1)], ob.F64, ob.DECIMATE, 2),
    # BASELINE configs[3] as stated: 2048 x 2048 x 256 planes, z chunk 64
    ("c4_u16_2048x256z_mean", [(ob.TIME, 0, 1, 1), (ob.SPACE, 256, 64, 1),
                               (ob.SPACE, 2048, 256, 1), (ob.SPACE, 2048, 256, 1)],
     ob.U16, ob.MEAN, 256),
]


def digest_frame(key, dt, h, w, seed, i):
    """Input frame i of a digest case: splitmix64 from the case's seed, with
    edge values sprinkled in for the *_specials cases."""
    fr = ob.synthetic_frames(dt, 1, h, w, seed + i)
    if key.endswith("_specials"):
        fr = with_specials(fr, dt, seed + i + 7919, frac=0.05)
    return fr[0]


def frame_digest(img, dt):
    """sha256 of a level frame; float NaNs canonicalised first (their sign
    and payload are not part of the parity contract: tests/helpers.py)."""
    a = np.ascontiguousarray(img)
    if dt in (ob.F32, ob.F64):
        a = a.copy()
        a[np.isnan(a)] = np.nan
    return hashlib.sha256(a.tobytes()).hexdigest()


def digest_seed(key):
    return int(hashlib.sha256(key.encode()).hexdigest()[:12], 16)


def write_metadata():
    import ctypes as C
    R = ob.ref()
    R.ref_ds_metadata.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
    R.ref_ds_metadata.restype = C.c_size_t
    R.ref_ds_method_name.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
    R.ref_ds_method_name.restype = C.c_size_t
    out = {}
    dims = [(ob.TIME, 0, 5, 1), (ob.SPACE, 10, 5, 1), (ob.SPACE, 10, 5, 1)]
    for m in range(4):
        ds = ob.OracleDownsampler(dims, ob.U16, m, 0, use_ref=True)
        buf = C.create_string_buffer(4096)
        n = R.ref_ds_metadata(ds.h, buf, 4096)
        assert n < 4096
        name = C.create_string_buffer(64)
        R.ref_ds_method_name(ds.h, name, 64)
        out[str(m)] = {"method_name": name.value.decode(), "metadata": buf.value.decode()}
    with open(os.path.join(HERE, "metadata.json"), "w") as f:
        json.dump(out, f, indent=1)


def main():
    if not ob.ref_available():
        sys.exit("oracle/_ref/libaqzref.so missing: run `make -C oracle ref` first")
    write_metadata()
    if sys.argv[1:] == ["metadata"]:
        return
    if sys.argv[1:] != ["digests"]:
        write_small()
    write_digests()


def write_small():
    arrays = {}
    for key, dims, dt, m, frames in cascade_cases():
        ds = ob.OracleDownsampler(dims, dt, m, 0, use_ref=True)
        arrays[f"{key}/in"] = frames
        arrays[f"{key}/dims"] = np.array(dims, dtype=np.int64)
        arrays[f"{key}/meta"] = np.array([dt, m], dtype=np.int64)
        for i in range(frames.shape[0]):
            ds.add_frame(frames[i])
            for lvl in range(1, ds.n_levels()):
                img = ds.take_frame(lvl)
                if img is not None:
                    arrays[f"{key}/out/{i}/{lvl}"] = img
    np.savez_compressed(os.path.join(HERE, "cascade_small.npz"), **arrays)

    tiles = {}
    for key, dims, dt in TILE_CASES:
        od = ob.OracleDims(dims, dt, use_ref=True)
        h, w = dims[-2][1], dims[-1][1]
        F = od.frames_per_chunk_layer()
        frames = ob.synthetic_frames(dt, F, h, w, digest_seed(key))
        frames[1] = 0  # an all-zero frame
        layer, flags = od.new_layer()
        for fid in range(F):
            od.write_frame_to_chunks(fid, frames[fid], layer, flags)
        tiles[f"{key}/in"] = frames
        tiles[f"{key}/dims"] = np.array(dims, dtype=np.int64)
        tiles[f"{key}/dtype"] = np.array([dt], dtype=np.int64)
        tiles[f"{key}/layer"] = layer
        tiles[f"{key}/has_data"] = flags
    np.savez_compressed(os.path.join(HERE, "tile_split.npz"), **tiles)


def write_digests():
    digests = {}
    for key, dims, dt, m, n in DIGEST_CASES:
        ds = ob.OracleDownsampler(dims, dt, m, 0, use_ref=True)
        h, w = dims[-2][1], dims[-1][1]
        seed = digest_seed(key)
        rec = {"dims": dims, "dtype": dt, "method": m, "frames": n, "seed": seed,
               "specials": key.endswith("_specials"),
               "levels": [ds.level_dims(lvl) for lvl in range(ds.n_levels())], "out": []}
        for i in range(n):
            fr = digest_frame(key, dt, h, w, seed, i)
            ds.add_frame(fr)
            for lvl in range(1, ds.n_levels()):
                img = ds.take_frame(lvl)
                if img is not None:
                    rec["out"].append([i, lvl, frame_digest(img, dt)])
        digests[key] = rec
        print(key, len(rec["out"]), "level frames", flush=True)
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(digests, f, indent=1)


if __name__ == "__main__":
    main()
