"""CPU suite, part 2: the C-ABI library loads and exports every entry point
include/aqz_gpu.h declares, and its host-side restatement of the chunk
lattice / level geometry (which drives the kernels' addressing) matches the
oracle and the compiled reference.  No GPU compute is called here."""
import os
import re

import numpy as np
import pytest

import aqz
import oracle_bindings as ob

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(REPO, "include", h) for h in ("aqz_gpu.h", "aqz_gpu_bench.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(aqz_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    L = aqz.lib()
    names = declared_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # the binding wires every declared entry point
    import inspect
    src = inspect.getsource(aqz.lib)
    assert all(f'"{n}"' in src for n in names)


def test_library_is_gfx950_and_in_tree():
    assert aqz.LIB_PATH.startswith(os.path.join(REPO, "acquire-zarr_amd"))
    blob = open(aqz.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_status_messages_and_version():
    L = aqz.lib()
    assert L.aqz_version() == b"0.1.0"
    assert L.aqz_status_message(0) == b"Success"
    assert L.aqz_status_message(12) == b"Attempted write beyond array boundary"
    assert aqz.device_count() >= 0


def test_invalid_settings_map_to_status_codes():
    with pytest.raises(aqz.AqzError) as e:
        aqz.Dims([(ob.SPACE, 10, 5, 1)], ob.U16)
    assert e.value.status == 9
    with pytest.raises(aqz.AqzError) as e:
        aqz.Dims([(ob.TIME, 0, 1, 1), (ob.CHANNEL, 3, 1, 1), (ob.SPACE, 10, 5, 1)], ob.U16)
    assert e.value.status == 9
    with pytest.raises(aqz.AqzError) as e:
        aqz.Dims([(ob.TIME, 0, 1, 1), (ob.SPACE, 10, 5, 1), (ob.SPACE, 10, 5, 1)], 10)
    assert e.value.status == 1
    with pytest.raises(aqz.AqzError) as e:  # dim 0 moved away
        aqz.Dims([(ob.TIME, 0, 1, 1), (ob.SPACE, 4, 2, 1), (ob.SPACE, 10, 5, 1),
                  (ob.SPACE, 10, 5, 1)], ob.U16, storage_order=[1, 0, 2, 3])
    assert e.value.status == 9


def _random_dims(rng):
    nd = int(rng.integers(3, 6))
    dims = [(ob.TIME, int(rng.integers(0, 3)) * 4, int(rng.integers(1, 6)),
             int(rng.integers(1, 3)))]
    for _ in range(nd - 3):
        dims.append((int(rng.integers(0, 3)), int(rng.integers(1, 7)),
                     int(rng.integers(1, 4)), int(rng.integers(1, 3))))
    dims += [(ob.SPACE, int(rng.integers(1, 80)), int(rng.integers(1, 12)),
              int(rng.integers(1, 3))),
             (ob.SPACE, int(rng.integers(1, 80)), int(rng.integers(1, 12)),
              int(rng.integers(1, 3)))]
    return dims


def test_host_index_math_matches_oracle():
    rng = np.random.default_rng(11)
    for _ in range(150):
        dims = _random_dims(rng)
        dt = int(rng.integers(0, 10))
        a, o = aqz.Dims(dims, dt), ob.OracleDims(dims, dt)
        assert a.dims() == [tuple(d) for d in dims]
        assert a.bytes_per_chunk() == o.bytes_per_chunk()
        assert a.number_of_chunks_in_memory() == o.number_of_chunks_in_memory()
        assert a.frames_per_chunk_layer() == o.frames_per_chunk_layer()
        for fid in range(40):
            assert a.tile_group_offset(fid) == o.tile_group_offset(fid)
            assert a.chunk_internal_offset(fid) == o.chunk_internal_offset(fid)
            for d in range(len(dims) - 2):
                assert a.chunk_lattice_index(fid, d) == o.chunk_lattice_index(fid, d)
            assert a.transpose_frame_id(fid) == fid
        cps = int(np.prod([d[3] for d in dims]))
        nsh = int(np.prod([-(-(-(-d[1] // d[2])) // d[3]) for d in dims[1:]]))
        for c in range(min(cps * nsh, 200)):
            assert a.shard_index_for_chunk(c) == o.shard_index_for_chunk(c)
            assert a.shard_internal_index(c) == o.shard_internal_index(c)


def test_host_pyramid_levels_match_oracle():
    rng = np.random.default_rng(12)
    for _ in range(200):
        dims = _random_dims(rng)
        ml = int(rng.integers(0, 4))
        lv = aqz.pyramid_levels(dims, ml)
        od = ob.OracleDownsampler(dims, ob.U16, ob.MEAN, ml)
        assert len(lv) == od.n_levels()
        for l, d in enumerate(lv):
            assert [tuple(x) for x in d] == [tuple(x) for x in od.level_dims(l)]
    # 2-D arrays get the phantom singleton (array.dimensions.cpp:149-153)
    lv = aqz.pyramid_levels([(ob.SPACE, 64, 16, 1), (ob.SPACE, 64, 16, 1)])
    assert len(lv) == 3 and lv[0][0] == (ob.OTHER, 1, 1, 1)


@pytest.mark.skipif(not ob.ref_available(), reason="oracle/_ref not built")
def test_host_transposition_matches_reference():
    rng = np.random.default_rng(13)
    for _ in range(60):
        inner = [(ob.CHANNEL, int(rng.integers(1, 5)), 1, 1),
                 (ob.SPACE, int(rng.integers(1, 6)), int(rng.integers(1, 3)), 1),
                 (ob.OTHER, int(rng.integers(1, 4)), 1, 1)]
        dims = [(ob.TIME, int(rng.integers(0, 2)) * 3, int(rng.integers(1, 3)), 1)] + inner + \
               [(ob.SPACE, 12, 4, 1), (ob.SPACE, 8, 4, 1)]
        perm = [0] + [1 + int(i) for i in rng.permutation(3)] + [4, 5]
        a = aqz.Dims(dims, ob.U16, storage_order=perm)
        r = ob.OracleDims(dims, ob.U16, use_ref=True, order=perm)
        n = 60 if dims[0][1] == 0 else int(np.prod([d[1] for d in dims[:-2]]))
        for fid in range(n):
            assert a.transpose_frame_id(fid) == r.transpose_frame_id(fid)
            assert a.tile_group_offset(a.transpose_frame_id(fid)) == \
                r.tile_group_offset(r.transpose_frame_id(fid))


@pytest.mark.skipif(not ob.ref_available(), reason="oracle/_ref not built")
def test_dim1_banding_geometry_matches_reference():
    """supports_dim1_banding / dim1_band_count / frames_per_dim1_band /
    chunks_per_dim1_band (array.dimensions.cpp:344-373)."""
    import ctypes as C
    R = ob.ref()
    R.ref_dims_dim1_banding.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
    rng = np.random.default_rng(14)
    seen = set()
    for _ in range(150):
        dims = _random_dims(rng)
        if rng.integers(0, 2):
            dims[0] = (dims[0][0], dims[0][1], 1, dims[0][3])  # append chunk 1
        a = aqz.Dims(dims, ob.U16)
        r = ob.OracleDims(dims, ob.U16, use_ref=True)
        s, n, f, c = C.c_int(), C.c_uint32(), C.c_uint64(), C.c_uint32()
        R.ref_dims_dim1_banding(r.h, C.byref(s), C.byref(n), C.byref(f), C.byref(c))
        got = a.dim1_banding()
        assert got == (bool(s.value), n.value, f.value, c.value), dims
        seen.add(got[0])
    assert seen == {True, False}
    # C4 (BASELINE configs[3]): 4 z bands of 64 planes, 64 chunks each
    c4 = [(ob.TIME, 0, 1, 1), (ob.SPACE, 256, 64, 1), (ob.SPACE, 2048, 256, 1),
          (ob.SPACE, 2048, 256, 1)]
    assert aqz.Dims(c4, ob.U16).dim1_banding() == (True, 4, 64, 64)


@pytest.mark.skipif(not ob.ref_available(), reason="oracle/_ref not built")
def test_shard_skip_lists_match_reference():
    """aqz_dims_shard_geometry and aqz_dims_skipped_internal_indices (what
    the binding's ShardRouter skips on a layer's last unit) against the
    compiled reference's chunks_per_shard / number_of_shards /
    chunk_layers_per_shard and skipped_internal_indices_for_shard_layer
    (array.dimensions.cpp:376-453), over random ragged shapes."""
    import ctypes as C
    R = ob.ref()
    u32p = C.POINTER(C.c_uint32)
    R.ref_dims_shard_geometry.argtypes = [C.c_void_p, u32p, u32p, u32p]
    R.ref_dims_skipped_internal_indices.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32,
                                                    u32p, C.c_size_t]
    R.ref_dims_skipped_internal_indices.restype = C.c_size_t
    rng = np.random.default_rng(15)
    nonempty = 0
    for _ in range(120):
        dims = _random_dims(rng)
        a = aqz.Dims(dims, ob.U16)
        r = ob.OracleDims(dims, ob.U16, use_ref=True)
        g = [C.c_uint32() for _ in range(3)]
        R.ref_dims_shard_geometry(r.h, *[C.byref(x) for x in g])
        assert a.shard_geometry() == tuple(x.value for x in g), dims
        cps, ns, lps = a.shard_geometry()
        buf = (C.c_uint32 * max(1, cps))()
        for shard in range(ns):
            for layer in range(max(1, lps)):
                n = R.ref_dims_skipped_internal_indices(r.h, shard, layer, buf, cps)
                got = a.skipped_internal_indices(shard, layer)
                assert got == list(buf[:n]), (dims, shard, layer)
                nonempty += bool(got)
    assert nonempty > 0  # some shapes have ragged padding
    with pytest.raises(aqz.AqzError):
        aqz.Dims(dims, ob.U16).skipped_internal_indices(ns, 0)


def test_memory_estimate_counts_the_rings():
    """aqz_stage_estimate_memory (no GPU): the chunk-layer rings dominate;
    for C2 as benched's level-0 geometry, 3 slots x 64 chunks x 8 MiB."""
    c2 = [(ob.TIME, 0, 64, 1), (ob.SPACE, 2048, 256, 1), (ob.SPACE, 2048, 256, 1)]
    m = aqz.estimate_memory(c2, ob.U16, ob.MEAN, max_batch_frames=128, layer_slots=2)
    ring0 = 3 * 64 * 256 * 256 * 64 * 2
    lv = aqz.pyramid_levels(c2)
    rings = sum(3 * (-(-d[-1][1] // 256)) * (-(-d[-2][1] // 256)) * 256 * 256 * 64 * 2
                for d in lv)
    assert rings >= ring0
    staging = 2 * 128 * 2048 * 2048 * 2
    assert rings + staging <= m["device_bytes"] <= rings + staging + (1 << 30)
    assert m["pinned_bytes"] >= staging
    big = aqz.estimate_memory(c2, ob.U16, ob.MEAN, max_batch_frames=128, layer_slots=4)
    assert big["device_bytes"] > m["device_bytes"]


def test_memory_estimate_counts_the_ring_arena():
    """Rings of >= 256 MiB in all are packed (64 KiB aligned) into one arena
    of 2 MiB virtual-memory pieces: the estimate adds that rounding, which
    the per-level allocations (bench ring_malloc_flags 0x10000) do not have;
    smaller rings stay per level either way."""
    plain = dict(ring_malloc_flags=0x10000)
    # ragged 100-px chunks: ring sizes are not multiples of 64 KiB
    big = [(ob.TIME, 0, 64, 1), (ob.SPACE, 2000, 100, 1), (ob.SPACE, 2000, 100, 1)]
    a = aqz.estimate_memory(big, ob.U16, ob.MEAN, max_batch_frames=64, layer_slots=3)
    b = aqz.estimate_memory(big, ob.U16, ob.MEAN, max_batch_frames=64, layer_slots=3, **plain)
    n_levels = len(aqz.pyramid_levels(big))
    assert 0 < a["device_bytes"] - b["device_bytes"] < (2 << 20) + n_levels * (64 << 10)
    small = [(ob.TIME, 0, 4, 1), (ob.SPACE, 512, 128, 1), (ob.SPACE, 512, 128, 1)]
    assert (aqz.estimate_memory(small, ob.U16, ob.MEAN) ==
            aqz.estimate_memory(small, ob.U16, ob.MEAN, **plain))
