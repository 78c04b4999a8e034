"""GPU: the hand-off side of the boundary.

* dim-1 bands (Array::flush_completed_bands_, array.cpp:873-908): a band's
  chunk range is handed off as soon as its frames are written, before its
  layer is complete, and equals the oracle's chunks;
* memory accounting (aqz_stage_memory_usage <= aqz_stage_estimate_memory);
* device sources produced on another stream (aqz_stage_wait_stream): the
  stage orders its reads after torch's queued work with no host sync.
"""
import numpy as np
import pytest

from helpers import assert_same_pixels, expected_stage_layers
from oracle_bindings import MEAN, SPACE, TIME, U16, synthetic_frames

pytestmark = pytest.mark.gpu


def test_stage_band_handoff_matches_oracle(gpu):
    # C4's structure at a small size: z 64 in 16-plane chunks -> 4 bands at
    # level 0, 2 at level 1 (z 32), 1 at level 2 (z 16)
    dims = [(TIME, 0, 1, 1), (SPACE, 64, 16, 1), (SPACE, 256, 64, 1), (SPACE, 256, 64, 1)]
    frames = synthetic_frames(U16, 64, 256, 256, 91)
    frames[20:24] = 0  # a band with some all-zero chunks
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    st = gpu.Stage(dims, U16, MEAN, max_batch_frames=8)
    L = st.n_levels()
    geo = [st.band_geometry(l) for l in range(L)]
    assert geo[0] == (True, 4, 16, 16)
    assert geo[1][:2] == (True, 2)
    lay = [st.layout(l) for l in range(L)]
    got = {}
    handed = [0] * L
    for b0 in range(0, 64, 8):
        st.append(np.ascontiguousarray(frames[b0:b0 + 8]))
        for l in range(L):
            ok, nb, fpb, cpb = geo[l]
            # the next band is not complete yet: refused
            if handed[l] < nb and st.frames_written(l) < (handed[l] + 1) * fpb:
                with pytest.raises(gpu.AqzError) as e:
                    st.copy_band_async(l, 0, handed[l], 0, 0)
                assert e.value.status == 3
            while handed[l] < nb and st.frames_written(l) >= (handed[l] + 1) * fpb:
                nbytes = cpb * lay[l]["bytes_per_chunk"]
                buf, hd = gpu.HostBuffer(nbytes), gpu.HostBuffer(cpb)
                st.copy_band_async(l, 0, handed[l], buf.ptr, nbytes, hd.ptr, cpb)
                got[(l, handed[l])] = (buf, hd)
                handed[l] += 1
    st.wait_copies()
    for l in range(L):
        ok, nb, fpb, cpb = geo[l]
        assert handed[l] == nb
        layer, flags = exp[(l, 0)]
        bpc = lay[l]["bytes_per_chunk"]
        for b in range(nb):
            buf, hd = got[(l, b)]
            assert_same_pixels(buf.array.copy(), layer[b * cpb * bpc:(b + 1) * cpb * bpc],
                               U16, f"L{l} band {b}")
            assert np.array_equal(hd.array, flags[b * cpb:(b + 1) * cpb]), (l, b)
    assert exp[(0, 0)][1][:16].any()  # has_data mixes 1s ...
    st.close()


def test_stage_band_handoff_ragged_dim1(gpu):
    """dim 1 not a multiple of its chunk (z 48 in 32-plane chunks): the
    trailing band holds 16 planes and is complete with its layer
    (flush_layer_remainder_, array.cpp:863-886), before any frame of the
    next layer arrives."""
    dims = [(TIME, 0, 1, 1), (SPACE, 48, 32, 1), (SPACE, 128, 64, 1), (SPACE, 128, 64, 1)]
    frames = synthetic_frames(U16, 96, 128, 128, 7)  # two timepoints
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    st = gpu.Stage(dims, U16, MEAN, max_batch_frames=8, layer_slots=3)
    L = st.n_levels()
    geo = [st.band_geometry(l) for l in range(L)]
    lay = [st.layout(l) for l in range(L)]
    assert geo[0][:3] == (True, 2, 32)
    got = {}
    nxt = [(0, 0)] * L  # (layer, band) to hand off next, per level
    for b0 in range(0, 96, 8):
        st.append(np.ascontiguousarray(frames[b0:b0 + 8]))
        for l in range(L):
            ok, nb, fpb, cpb = geo[l]
            F = lay[l]["frames_per_layer"]
            while True:
                layer, band = nxt[l]
                if (layer, 0) not in exp:
                    break
                end = layer * F + min((band + 1) * fpb, F)
                if st.frames_written(l) < end:
                    with pytest.raises(gpu.AqzError) as e:
                        st.copy_band_async(l, layer, band, 0, 0)
                    assert e.value.status == 3
                    break
                nbytes = cpb * lay[l]["bytes_per_chunk"]
                buf, hd = gpu.HostBuffer(nbytes), gpu.HostBuffer(cpb)
                st.copy_band_async(l, layer, band, buf.ptr, nbytes, hd.ptr, cpb)
                got[(l, layer, band)] = (buf, hd)
                nxt[l] = (layer, band + 1) if band + 1 < nb else (layer + 1, 0)
        # the trailing band of layer 0 leaves with the layer's last frame
        if b0 + 8 == 48:
            assert (0, 0, 1) in got
        st.wait_copies()
    for (l, layer), (buf, flags) in exp.items():
        ok, nb, fpb, cpb = geo[l]
        bpc = lay[l]["bytes_per_chunk"]
        for b in range(nb):
            hb, hd = got[(l, layer, b)]
            assert_same_pixels(hb.array.copy(), buf[b * cpb * bpc:(b + 1) * cpb * bpc],
                               U16, f"L{l} layer {layer} band {b}")
            assert np.array_equal(hd.array, flags[b * cpb:(b + 1) * cpb]), (l, layer, b)
    st.close()


def test_stage_band_geometry_without_banding(gpu):
    dims = [(TIME, 0, 4, 1), (SPACE, 64, 16, 1), (SPACE, 64, 16, 1)]
    st = gpu.Stage(dims, U16, MEAN)
    ok, nb, fpb, cpb = st.band_geometry(0)
    assert (ok, nb, fpb, cpb) == (False, 1, 4, st.layout(0)["chunks_per_layer"])
    st.close()


def test_stage_memory_usage_within_estimate(gpu):
    dims = [(TIME, 0, 16, 1), (SPACE, 1024, 256, 1), (SPACE, 1024, 256, 1)]
    est = gpu.estimate_memory(dims, U16, MEAN, max_batch_frames=16, layer_slots=2)
    st = gpu.Stage(dims, U16, MEAN, max_batch_frames=16, layer_slots=2)
    m0 = st.memory_usage()
    lay = [st.layout(l) for l in range(st.n_levels())]
    rings = sum(x["chunk_pitch"] * x["chunks_per_layer"] * x["layer_slots"] for x in lay)
    assert rings <= m0["device_bytes"] <= est["device_bytes"]
    frames = synthetic_frames(U16, 16, 1024, 1024, 3)
    st.append(frames)  # pageable: staging buffers appear
    st.synchronize()
    m1 = st.memory_usage()
    assert m1["pinned_bytes"] > m0["pinned_bytes"]
    assert m1["device_bytes"] > m0["device_bytes"]
    assert m1["device_bytes"] <= est["device_bytes"]
    assert m1["pinned_bytes"] <= est["pinned_bytes"]
    st.close()


def test_stage_append_cuda_tensor_from_side_stream(gpu):
    """Frames written by torch on a side stream and appended at once (no
    synchronize, the tensor dropped right after): the stage's stream waits
    for torch's work, and the binding keeps the tensor alive until read."""
    import torch
    dims = [(TIME, 0, 4, 1), (SPACE, 512, 128, 1), (SPACE, 512, 128, 1)]
    frames = synthetic_frames(U16, 8, 512, 512, 17)
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    src = torch.from_numpy(frames.view(np.int16)).cuda()
    torch.cuda.synchronize()
    st = gpu.Stage(dims, U16, MEAN, max_batch_frames=4, layer_slots=4)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        for b0 in (0, 4):
            # a long queue of torch work ahead of the copy the stage reads
            junk = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
            for _ in range(20):
                junk.add_(1)
            t = src[b0:b0 + 4].clone()
            st.append(t)
            del t, junk
    st.finalize()
    for (l, layer), (buf, flags) in exp.items():
        got, gflags = st.copy_layer(l, layer)
        assert_same_pixels(got, buf, U16, f"L{l}")
        assert np.array_equal(gflags, flags)
    assert not st._held  # released once consumed
    st.close()


class Replay:
    def __init__(self, log, summary, got, padding, rollovers):
        self.log, self.summary, self.got = log, summary, got
        self.padding, self.rollovers = padding, rollovers


def _run_replay(tmp_path, dims, dtype, method, frames, batch, slots, codec=(0, 0, 0),
                copy_threads=4, pool_threads=4, device=0, synth=0, n_frames=None,
                placement_tries=0, record=True, z_slabs=1, level0=None):
    """tests/native/handoff_replay: the binding's hand-off
    (integration/aqz_handoff.hh, what GpuMultiscaleArray runs) over the C
    ABI; every unit goes through the shipped ShardRouter (what GpuArray
    runs) into a recording ShardWriter that does GpuArray's per-chunk copy
    on a thread pool.  Returns a Replay: the unit log, the summary, got =
    {(level, layer, chunk): (shard, internal, bytes, append-shard row)}, the
    ragged-padding skips [(level, layer, row, shard, internal)] and each
    level's rollover points (frames committed)."""
    import json
    import os
    import struct
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "handoff_replay")
    assert os.path.exists(exe), "make -C tests/native (built by __graft_entry__.build)"
    job, out = tmp_path / "job.bin", tmp_path / "out.bin"
    fb = frames[0].nbytes if frames is not None else None
    with open(job, "wb") as f:
        f.write(b"AQZ2" + struct.pack("<I", len(dims)))
        for d in dims:
            f.write(struct.pack("<iIII", *d))
        n = len(frames) if frames is not None else n_frames
        if fb is None:
            fb = dims[-1][1] * dims[-2][1] * {0: 1, 1: 2}[dtype]
        f.write(struct.pack("<iiIIiiiiIIIIIQQ", dtype, method, batch, slots, device, *codec,
                            copy_threads, pool_threads, synth, placement_tries, z_slabs, n, fb))
        if frames is not None:
            f.write(np.ascontiguousarray(frames).tobytes())
    env = dict(os.environ)
    if level0:  # force the level-0 side (default: the binding's choice)
        env["AQZ_REPLAY_LEVEL0"] = level0
    r = subprocess.run([exe, str(job), str(out) if record else "-"], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    log = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    summary = log[-1]
    assert summary["summary"] and summary["ok"], summary
    got, padding, rollovers = {}, [], []
    if record:
        b = out.read_bytes()
        assert b[:4] == b"AQZ4"
        (nl,), o = struct.unpack_from("<I", b, 4), 8
        for l in range(nl):
            (nrec,) = struct.unpack_from("<Q", b, o)
            o += 8
            for _ in range(nrec):
                layer, chunk, append, shard, internal, nb = struct.unpack_from("<QIIIIQ", b, o)
                o += 32
                if chunk == 0xFFFFFFFF:  # ragged padding of a shard
                    padding.append((l, layer, append, shard, internal))
                    continue
                key = (l, layer, chunk)
                assert key not in got, f"chunk handed to its shard twice: {key}"
                got[key] = (shard, internal, b[o:o + nb], append)
                o += nb
            (nr,) = struct.unpack_from("<Q", b, o)
            o += 8
            rollovers.append(list(struct.unpack_from(f"<{nr}Q", b, o)))
            o += 8 * nr
    return Replay(log[:-1], summary, got, padding, rollovers)


def _decode(codec, frame, bpc):
    from codec_helpers import blosc_zstd_decode, libblosc, libblosc_decode, oracle_decode, \
        zstd_decode
    if codec == 0:
        return frame
    if codec == 1:
        out = oracle_decode(frame)
        if libblosc():
            assert libblosc_decode(frame) == out
        return out
    if codec == 2:
        return libblosc_decode(frame) if libblosc() else blosc_zstd_decode(frame)
    return zstd_decode(frame, bpc)


def _check_replay(exp, fw, r, codec, st):
    """Every chunk of every oracle layer reached its shard exactly once:
    skipped iff the oracle's has_data is false, else bytes that decode to
    the oracle's chunk; units contiguous and in frame order per level; and
    the shard routing is the reference's (_check_routing)."""
    log, got = r.log, r.got
    per = {}
    for e in log:
        prev = per.setdefault(e["level"], [])
        assert e["first"] == sum(x["frames"] for x in prev), e  # contiguous, in order
        prev.append(e)
    for l, units in per.items():
        assert sum(u["frames"] for u in units) == fw[l]
        first_open = [i for i, u in enumerate(units) if not u["complete"]]
        assert not first_open or all(not u["complete"] for u in units[first_open[0]:])
    seen = set()
    for (l, layer), (buf, flags) in exp.items():
        bpc = st.layout(l)["bytes_per_chunk"]
        for c in range(len(flags)):
            key = (l, layer, c)
            assert key in got, f"chunk never reached its shard: {key}"
            seen.add(key)
            _, _, data, _ = got[key]
            if not flags[c]:
                assert len(data) == 0, f"{key}: a chunk without data must be skipped"
                continue
            assert len(data) > 0, f"{key}: a chunk with data was skipped"
            dec = _decode(codec[0], data, bpc)
            assert dec == buf[c * bpc:(c + 1) * bpc].tobytes(), f"{key}: decoded bytes differ"
    assert seen == set(got), sorted(set(got) - seen)[:5]
    _check_routing(r, fw, st)
    # what the live hand-off and its stages hold against the binding's
    # estimate (aqz_binding::estimate_memory, the drop-in's memory contract)
    sm = r.summary
    assert 0 < sm["host_bytes"] <= sm["estimate_host_bytes"], sm
    assert 0 < sm["device_bytes"] <= sm["estimate_device_bytes"], sm


def _check_routing(r, fw, st):
    """The shipped ShardRouter's routing against the reference's rules, per
    level: a chunk of layer k goes to append-shard row k // layers_per_shard
    at (shard_index_for_chunk, shard_internal_index) of chunk index
    (k mod layers_per_shard) * chunks_in_memory + slot (the compiled
    reference's ArrayDimensions when oracle/_ref is built,
    array.dimensions.cpp:393-548; compress_and_flush_data_, array.cpp:
    762-811); rollovers fall exactly where should_rollover_ says (every
    frames_per_layer * layers_per_shard committed frames, array.cpp:924-951);
    and in every completed row each shard's internal indices are written or
    skipped exactly once -- chunks, chunks without data and the ragged
    padding together (skipped_internal_indices_for_shard_layer,
    array.dimensions.cpp:424-453) -- so every shard's countdown completes."""
    import aqz
    from oracle_bindings import OracleDims, ref_available
    for l in range(st.n_levels()):
        ld = st.level_dims(l)
        ref = OracleDims(ld, U16, use_ref=ref_available())
        cps, ns, lps = aqz.Dims(ld, U16).shard_geometry()
        n_mem = ref.number_of_chunks_in_memory()
        F = ref.frames_per_chunk_layer()
        done_layers = fw[l] // F
        assert r.rollovers[l] == [k * F * lps for k in range(1, done_layers // lps + 1)], l
        rows = {}
        for (lv, layer, chunk), (shard, internal, _, append) in r.got.items():
            if lv != l:
                continue
            assert append == layer // lps, (l, layer, chunk, append)
            c = (layer % lps) * n_mem + chunk
            assert (shard, internal) == (ref.shard_index_for_chunk(c),
                                         ref.shard_internal_index(c)), (l, layer, chunk)
            rows.setdefault((append, shard), []).append(internal)
        for (lv, layer, append, shard, internal) in r.padding:
            if lv == l:  # complete layers, and the partial last one at close
                assert append == layer // lps and layer <= done_layers, (l, layer)
                rows.setdefault((append, shard), []).append(internal)
        for a in range(done_layers // lps):
            for s_ in range(ns):
                assert sorted(rows.get((a, s_), [])) == list(range(cps)), (l, a, s_)


REPLAY_CASES = {
    # dim-1 bands: 3-D, chunk 1 on the append dim, z chunk 16 of 64
    "banded-3d": ([(TIME, 0, 1, 1), (SPACE, 64, 16, 1), (SPACE, 256, 64, 1),
                   (SPACE, 256, 64, 1)], 2 * 64 + 24, 8),
    # append shards of 2 layers over 5 layers (two rollovers), banded, ragged
    # 3-chunk x and 5-chunk y in 2x2 shards (padding in the edge shards)
    "banded-rollover": ([(TIME, 0, 1, 2), (SPACE, 48, 16, 1), (SPACE, 300, 64, 2),
                         (SPACE, 192, 64, 2)], 5 * 48 + 10, 8),
    # ragged dim 1 (48 planes, 32-plane chunks): the trailing band holds 16
    # frames and is complete with its layer (array.cpp:884-886)
    "banded-ragged": ([(TIME, 0, 1, 1), (SPACE, 48, 32, 1), (SPACE, 256, 64, 2),
                       (SPACE, 192, 64, 2)], 3 * 48 + 20, 7),
    # 2-D, ragged tiles and a partial last layer; shards of 2 x 2 chunks
    "layers-2d-ragged": ([(TIME, 0, 4, 2), (SPACE, 300, 64, 2), (SPACE, 260, 64, 2)],
                         4 * 9 + 3, 5),
    # a bounded append dimension (10 frames in 4-frame chunks): the array is
    # full at close, its last layer holds 2 frames and padding
    "bounded-append": ([(TIME, 10, 4, 2), (SPACE, 300, 64, 2), (SPACE, 260, 64, 2)], 10, 3),
}
CODECS = {"raw": (0, 0, 0), "lz4-shuffle": (1, 5, 1), "blosc-zstd-bitshuffle": (2, 5, 2),
          "zstd-1": (3, 1, 0), "zstd-3": (3, 3, 0)}


@pytest.mark.parametrize("codec", sorted(CODECS))
@pytest.mark.parametrize("case", sorted(REPLAY_CASES))
def test_binding_handoff_replay(gpu, tmp_path, case, codec):
    """The reference-side binding's consumer path, replayed natively: frames
    batched into pinned double buffers by copy threads, asynchronous appends
    refilled after aqz_stage_wait_consumed, every unit -- a raw band / layer,
    or a layer compressed on the device and copied out once its compression
    finished -- handed to the sink in frame order with a lease on its host
    buffer, and every chunk copied into a vector on a pool thread as
    GpuArray::write_unit does before Shard::write_chunk.  Every chunk of every
    layer reaches its shard exactly once, at the shard and internal index
    ArrayDimensions gives (checked in the replay), skipped iff it has no
    data, and decodes to the oracle's chunk (MultiscaleArray::write_frame,
    multiscale.array.cpp:57-74, 291-325; Array::dispatch_chunk_job_,
    array.cpp:664-760)."""
    from codec_helpers import libzstd
    if CODECS[codec][0] in (2, 3) and libzstd() is None:
        pytest.skip("no libzstd to decode with")
    dims, n, batch = REPLAY_CASES[case]
    h, w = dims[-2][1], dims[-1][1]
    frames = synthetic_frames(U16, n, h, w, 61 + n)
    if CODECS[codec][0]:
        # compressible: keep the low bits only, with all-zero frames mixed in
        frames &= 0x00ff
        frames[5:9] = 0
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    r = _run_replay(tmp_path, dims, U16, MEAN, frames, batch, 2, codec=CODECS[codec])
    # a raw hand-off splits level 0 on the host (the binding's choice)
    assert r.summary["level0_split"] == ("device" if CODECS[codec][0] else "host")
    st = gpu.Stage(dims, U16, MEAN)
    if case.startswith("banded") and not CODECS[codec][0]:
        assert len([e for e in r.log if e["level"] == 0]) > len(
            {k[1] for k in exp if k[0] == 0})  # bands, not layers
    _check_replay(exp, fw, r, CODECS[codec], st)
    st.close()


@pytest.mark.parametrize("codec", ["lz4-shuffle", "zstd-1", "raw"])
@pytest.mark.parametrize("slots", [1, 3])
def test_binding_handoff_replay_host_slots(gpu, tmp_path, codec, slots):
    """More (or fewer) host unit buffers per level than the stage has device
    layer slots: a compressed layer's device frame slot takes a newer layer
    as soon as its copy is issued, so the hand-off reads the entries at
    issue time; with one host buffer every unit waits for the previous
    unit's writer jobs (the lease)."""
    from codec_helpers import libzstd
    if CODECS[codec][0] in (2, 3) and libzstd() is None:
        pytest.skip("no libzstd to decode with")
    dims, n, batch = REPLAY_CASES["layers-2d-ragged"]
    frames = synthetic_frames(U16, n, dims[-2][1], dims[-1][1], 7 * slots) & 0x0fff
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    r = _run_replay(tmp_path, dims, U16, MEAN, frames, batch, slots, codec=CODECS[codec],
                    pool_threads=3)
    st = gpu.Stage(dims, U16, MEAN)
    _check_replay(exp, fw, r, CODECS[codec], st)
    st.close()


@pytest.mark.parametrize("codec", ["raw", "lz4-shuffle", "zstd-1"])
@pytest.mark.parametrize("slabs,tail", [(2, 0), (2, 37), (4, 0), (4, 21), (3, 50)])
def test_binding_z_slabs(gpu, tmp_path, codec, slabs, tail):
    """AQZ_Z_SLABS: one multiscale volume stream over N stages (here all on
    device 0; on a node, one GPU each), stage r receiving z slab r of every
    stack.  Each unit is assembled in one stage (round robin over layers)
    from the others' frames by aqz_stage_import_frames (peer reads over
    xGMI between GPUs) and handed off from there -- raw or compressed on
    that device.  A partial last stack (tail planes) leaves the unwritten
    frames zero.  Every chunk reaches its shard once and decodes to the
    single-stream oracle's chunk."""
    from codec_helpers import libzstd
    if CODECS[codec][0] in (2, 3) and libzstd() is None:
        pytest.skip("no libzstd to decode with")
    # z 64 -> 32 -> 16 -> 16 (xy 256 -> 32), z chunk 16: slabs align to 4
    dims = [(TIME, 0, 1, 1), (SPACE, 64, 16, 1), (SPACE, 256, 64, 2), (SPACE, 256, 64, 2)]
    n = 2 * 64 + tail
    frames = synthetic_frames(U16, n, 256, 256, 71 + slabs + tail) & 0x0fff
    frames[70:75] = 0
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    r = _run_replay(tmp_path, dims, U16, MEAN, frames, 8, 3, codec=CODECS[codec],
                    z_slabs=slabs)
    st = gpu.Stage(dims, U16, MEAN)
    _check_replay(exp, fw, r, CODECS[codec], st)
    st.close()


@pytest.mark.parametrize("case", sorted(REPLAY_CASES))
def test_binding_handoff_replay_level0_on_device(gpu, tmp_path, case):
    """The raw hand-off with level 0 split on the device and copied D2H (the
    path a compressed hand-off keeps for level 0, and the raw one before the
    host split): the same units, chunks and routing as the host split."""
    dims, n, batch = REPLAY_CASES[case]
    frames = synthetic_frames(U16, n, dims[-2][1], dims[-1][1], 83 + n)
    frames[5:9] = 0
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    r = _run_replay(tmp_path, dims, U16, MEAN, frames, batch, 2, level0="device")
    assert r.summary["level0_split"] == "device"
    st = gpu.Stage(dims, U16, MEAN)
    _check_replay(exp, fw, r, CODECS["raw"], st)
    st.close()


@pytest.mark.parametrize("copy_threads", [1, 3])
def test_binding_handoff_replay_host_split_frames_small_and_large(gpu, tmp_path, copy_threads):
    """The host split in the copy pass: frames under 1 MiB are copied and
    split by the consumer thread alone, larger ones by row ranges over the
    copy threads (each thread's rows into the same unit buffer); a ragged
    dim-1 band clears the slot a full band left (padding positions), and
    close zero-fills the unwritten frames of level 0's last layer."""
    dims = [(TIME, 0, 1, 1), (SPACE, 20, 8, 1)]
    n = 2 * 20 + 11  # two layers and a partial third; bands of 8, 8, 4 planes
    frames = synthetic_frames(U16, n, 1000, 640, 97 + copy_threads)  # 1.28 MB frames
    frames[30:33] = 0
    for fr, batch in ((frames, 6), (np.ascontiguousarray(frames[:, :300, :256]), 5)):
        d = dims[:2] + [(SPACE, fr.shape[1], 128, 2), (SPACE, fr.shape[2], 128, 2)]
        e, f, _ = expected_stage_layers(d, U16, MEAN, fr)
        r = _run_replay(tmp_path, d, U16, MEAN, fr, batch, 2, copy_threads=copy_threads)
        assert r.summary["level0_split"] == "host"
        st = gpu.Stage(d, U16, MEAN)
        _check_replay(e, f, r, CODECS["raw"], st)
        st.close()
