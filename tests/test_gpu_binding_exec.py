"""GPU: the shipped drop-in binding itself, executed.

oracle/_ref/binding_exec (tests/native/binding_exec.cpp, built by
`make -C oracle binding` where /root/reference exists) compiles
integration/multiscale.array.gpu.cpp unchanged -- GpuMultiscaleArray's
constructor, write_frame, memory_usage and close_, GpuArray's write_unit /
commit_unit / dispatch_bytes_job_ / rollover, make_gpu_multiscale_array,
gpu_slab_plan and estimate_gpu_array_memory -- over the reference's own
ArrayConfig, ArrayDimensions, Downsampler and ThreadPool (compiled from its
sources) and over test doubles of Array / MultiscaleArray / Shard
(tests/native/binding_doubles.hh: members restated from array.cpp,
multiscale.array.cpp and shard.cpp, whose definitions do not build here).
It streams frames through write_frame as ZarrStream_s does and finalizes.

Checked: every chunk of every level reaches its shard double exactly once
and decodes to the oracle's chunk (MultiscaleArray::write_frame,
multiscale.array.cpp:57-74, 291-325), skipped iff it has no data, at the
reference's shard routing; rollovers where should_rollover_ puts them
(array.cpp:924-951) with zarr.json rewritten at each; each level's frame
counters at close as Array::write_frame leaves them (array.cpp:196-219) with
nothing left for close_ to flush; every completed row's shards finished
their countdown; write_frame's refusals; memory_usage / device memory within
estimate_gpu_array_memory.
"""
import json
import os
import struct
import subprocess

import pytest

from helpers import expected_stage_layers
from oracle_bindings import F32, I16, MAX, MEAN, MIN, SPACE, TIME, U8, U16, synthetic_frames
from test_gpu_handoff import CODECS, REPLAY_CASES, Replay, _check_routing, _decode

pytestmark = pytest.mark.gpu

# BINDING_EXEC: another build of the harness (tools/binding_mutants.sh runs
# this file against deliberately broken bindings, each of which must fail)
EXE = os.environ.get("BINDING_EXEC") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "..", "oracle", "_ref", "binding_exec")


def _run_exec(tmp_path, dims, frames, batch, slots, codec=(0, 0, 0), pool_threads=4,
              z_slabs=1, dtype=U16, method=MEAN):
    """Run the binding on `frames`; batch 0 = through make_gpu_multiscale_array."""
    assert os.path.exists(EXE), "make -C oracle binding (built by __graft_entry__.build)"
    job, out = tmp_path / "job.bin", tmp_path / "out.bin"
    fb = frames[0].nbytes
    with open(job, "wb") as f:
        f.write(b"AQZ2" + struct.pack("<I", len(dims)))
        for d in dims:
            f.write(struct.pack("<iIII", *d))
        f.write(struct.pack("<iiIIiiiiIIIIIQQ", dtype, method, batch, slots, 0, *codec, 0,
                            pool_threads, 0, 0, z_slabs, len(frames), fb))
        f.write(frames.tobytes())
    # BINDING_EXEC_PREFIX: a launcher that execs the harness before it
    # touches the GPU (tools/binding_sanitize.sh: setarch -R for TSan)
    pre = os.environ.get("BINDING_EXEC_PREFIX", "").split()
    env = dict(os.environ)
    # where a stalled run is (phase, frames, chunks), every 10 s
    prog = tmp_path / "progress.txt"
    env.setdefault("BINDING_EXEC_PROGRESS", str(prog))
    try:
        r = subprocess.run(pre + [EXE, str(job), str(out)], capture_output=True, text=True,
                           timeout=float(os.environ.get("BINDING_EXEC_TIMEOUT", "240")),
                           env=env)
    except subprocess.TimeoutExpired as e:
        where = prog.read_text() if prog.exists() else "(no progress file)"
        raise AssertionError(f"binding_exec stalled: {where}\nstderr: {e.stderr}") from None
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-3000:] + r.stderr[-3000:]
    summary = lines[-1]
    assert summary["ok"] and not summary["errors"], summary
    got, padding, rollovers = {}, [], []
    b = out.read_bytes()
    assert b[:4] == b"AQZ4"
    (nl,), o = struct.unpack_from("<I", b, 4), 8
    for l in range(nl):
        (nrec,) = struct.unpack_from("<Q", b, o)
        o += 8
        for _ in range(nrec):
            layer, chunk, append, shard, internal, nb = struct.unpack_from("<QIIIIQ", b, o)
            o += 32
            if chunk == 0xFFFFFFFF:
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
    return Replay([], summary, got, padding, rollovers)


def _check_exec(exp, fw, r, codec, st, dtype=U16):
    got = r.got
    seen = set()
    for (l, layer), (buf, flags) in exp.items():
        bpc = st.layout(l)["bytes_per_chunk"]
        for c in range(len(flags)):
            key = (l, layer, c)
            assert key in got, f"chunk never reached its shard: {key}"
            seen.add(key)
            data = got[key][2]
            if not flags[c]:
                assert len(data) == 0, f"{key}: a chunk without data must be skipped"
                continue
            assert len(data) > 0, f"{key}: a chunk with data was skipped"
            assert _decode(codec[0], data, bpc) == buf[c * bpc:(c + 1) * bpc].tobytes(), key
    assert seen == set(got), sorted(set(got) - seen)[:5]
    _check_routing(r, fw, st)
    sm = r.summary
    assert sm["n_levels"] == st.n_levels()
    for e in sm["levels"]:
        l = e["level"]
        fbl = st.layout(l)["frame_bytes"]
        assert fbl % {U8: 1, U16: 2, I16: 2, F32: 4}[dtype] == 0
        assert e["frames_written"] == fw[l], e
        assert e["total_bytes_written"] == fw[l] * fbl, e
        assert e["last_frame_id"] == max(fw[l] - 1, 0), e
        assert e["bytes_to_flush"] == 0, e  # close_ has nothing to flush
        assert e["closed"], e
        assert e["rollovers"] == r.rollovers[l]
        assert e["append_chunk_index"] == len(e["rollovers"]), e
        # zarr.json at every rollover (array.cpp:209-212) and at close
        assert e["metadata_writes"] == len(e["rollovers"]) + (1 if fw[l] else 0), e
    assert sm["group_metadata_writes"] == 1
    # host memory (the base's CPU chunk buffers are never allocated: 0)
    assert 0 < sm["memory_usage_mid"] <= sm["estimate_host_bytes"], sm
    assert 0 < sm["memory_usage_end"] <= sm["estimate_host_bytes"], sm
    assert 0 < sm["device_memory_usage"] <= sm["estimate_device_bytes"], sm


@pytest.mark.parametrize("codec", ["raw", "lz4-shuffle", "zstd-1"])
@pytest.mark.parametrize("case", sorted(REPLAY_CASES))
def test_binding_executes(gpu, tmp_path, case, codec):
    """The binding's constructor, write_frame and close_ over every replay
    geometry: dim-1 bands, two rollovers, ragged bands and tiles, a bounded
    append dimension filled to the last frame (and one more refused)."""
    from codec_helpers import libzstd
    if CODECS[codec][0] in (2, 3) and libzstd() is None:
        pytest.skip("no libzstd to decode with")
    dims, n, batch = REPLAY_CASES[case]
    frames = synthetic_frames(U16, n, dims[-2][1], dims[-1][1], 131 + n)
    if CODECS[codec][0]:
        frames &= 0x00ff
    frames[5:9] = 0
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    r = _run_exec(tmp_path, dims, frames, batch, 2, codec=CODECS[codec])
    assert r.summary["oob_probed"] == (dims[0][1] > 0)
    st = gpu.Stage(dims, U16, MEAN)
    _check_exec(exp, fw, r, CODECS[codec], st)
    st.close()


@pytest.mark.parametrize("codec", ["raw", "zstd-1"])
def test_binding_executes_through_the_hook(gpu, tmp_path, codec):
    """make_gpu_multiscale_array, as configure_array_ calls it: the default
    batch (64 frames) and host slots, one pool thread (the binding then runs
    every chunk job inline, execute_job_with_retry)."""
    from codec_helpers import libzstd
    if CODECS[codec][0] in (2, 3) and libzstd() is None:
        pytest.skip("no libzstd to decode with")
    dims, n, _ = REPLAY_CASES["banded-rollover"]
    frames = synthetic_frames(U16, n, dims[-2][1], dims[-1][1], 17) & 0x0fff
    frames[40:44] = 0
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    r = _run_exec(tmp_path, dims, frames, 0, 0, codec=CODECS[codec], pool_threads=1)
    assert r.summary["factory"]
    st = gpu.Stage(dims, U16, MEAN)
    _check_exec(exp, fw, r, CODECS[codec], st)
    st.close()


@pytest.mark.parametrize("slabs", [2, 4])
def test_binding_executes_z_slabs(gpu, tmp_path, slabs):
    """AQZ_Z_SLABS through the binding: gpu_slab_plan and one stage per slab
    (all on the one visible device here)."""
    dims = [(TIME, 0, 1, 1), (SPACE, 64, 16, 1), (SPACE, 256, 64, 2), (SPACE, 256, 64, 2)]
    frames = synthetic_frames(U16, 2 * 64 + 21, 256, 256, 5 + slabs) & 0x0fff
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    r = _run_exec(tmp_path, dims, frames, 8, 3, codec=CODECS["lz4-shuffle"], z_slabs=slabs)
    st = gpu.Stage(dims, U16, MEAN)
    _check_exec(exp, fw, r, CODECS["lz4-shuffle"], st)
    st.close()


@pytest.mark.parametrize("codec", ["raw", "lz4-shuffle"])
@pytest.mark.parametrize("dtype,method", [(U8, MAX), (I16, MIN), (F32, MEAN)],
                         ids=["u8-max", "i16-min", "f32-mean"])
def test_binding_executes_dtypes_and_methods(gpu, tmp_path, dtype, method, codec):
    """The settings' data type and downsampling method through the binding
    (ZarrArraySettings -> ArrayConfig -> aqz_array_desc)."""
    dims, n, batch = REPLAY_CASES["layers-2d-ragged"]
    frames = synthetic_frames(dtype, n, dims[-2][1], dims[-1][1], 29 + dtype)
    frames[5:9] = 0
    exp, fw, _ = expected_stage_layers(dims, dtype, method, frames)
    r = _run_exec(tmp_path, dims, frames, batch, 2, codec=CODECS[codec], dtype=dtype,
                  method=method)
    st = gpu.Stage(dims, dtype, method)
    _check_exec(exp, fw, r, CODECS[codec], st, dtype)
    st.close()


@pytest.mark.parametrize("codec", ["raw", "zstd-1"])
def test_binding_executes_c2_frames(gpu, tmp_path, codec):
    """C2's frames (u16 2048 x 2048, 256-px chunks) through the hook, with
    16-frame chunk layers in append shards of 2 layers: five full layers
    (two rollovers) and a partial sixth; 8 MiB frames, so the copy threads
    split each frame's rows between them."""
    from codec_helpers import libzstd
    if CODECS[codec][0] in (2, 3) and libzstd() is None:
        pytest.skip("no libzstd to decode with")
    dims = [(TIME, 0, 16, 2), (SPACE, 2048, 256, 1), (SPACE, 2048, 256, 1)]
    frames = synthetic_frames(U16, 5 * 16 + 7, 2048, 2048, 2) & 0x0fff
    frames[20:23] = 0
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    r = _run_exec(tmp_path, dims, frames, 0, 0, codec=CODECS[codec], pool_threads=8)
    assert r.summary["factory"] and [len(x) for x in r.rollovers][0] == 2
    st = gpu.Stage(dims, U16, MEAN)
    _check_exec(exp, fw, r, CODECS[codec], st)
    st.close()


@pytest.mark.parametrize("codec", ["raw", "lz4-shuffle"])
def test_binding_executes_xy_storage_order(gpu, tmp_path, codec, monkeypatch):
    """storage_dimension_order with X and Y swapped (ZarrArraySettings ->
    ArrayDimensions' target order and aqz_array_desc): a raw hand-off then
    keeps level 0 on the device (level0_on_host_for), and every stored frame
    is the acquired one transposed (array.cpp:488-504, 525-533).  The append
    dimension is bounded, as in the reference's own test_swap_xy: with an
    unbounded one and only X/Y permuted the reference's ArrayDimensions
    cannot be built (compute_transposition, array.dimensions.cpp:96-102:
    lookup_dims is 0 and `lookup_dims - 1` wraps; it faults), so no stream
    reaches the binding with that array."""
    import numpy as np
    acq = [(TIME, 16, 4, 2), (SPACE, 300, 64, 2), (SPACE, 260, 64, 2)]
    frames = synthetic_frames(U16, 16, 300, 260, 45)
    if CODECS[codec][0]:
        frames &= 0x00ff
    frames[5:9] = 0
    perm = [0, 2, 1]
    stored = np.ascontiguousarray(frames.transpose(0, 2, 1))
    exp, fw, _ = expected_stage_layers([acq[i] for i in perm], U16, MEAN, stored)
    monkeypatch.setenv("BINDING_EXEC_ORDER", "0,2,1")
    r = _run_exec(tmp_path, acq, frames, 5, 2, codec=CODECS[codec])
    st = gpu.Stage(acq, U16, MEAN, storage_order=perm)
    _check_exec(exp, fw, r, CODECS[codec], st)
    st.close()
