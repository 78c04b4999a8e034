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


def _run_replay(tmp_path, dims, dtype, method, frames, batch, slots):
    """tests/native/handoff_replay: the binding's hand-off
    (integration/aqz_handoff.hh, what GpuMultiscaleArray runs) over the C
    ABI with a recording sink.  Returns (commit log, {(level, layer): (bytes,
    has_data)})."""
    import json
    import os
    import struct
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "handoff_replay")
    assert os.path.exists(exe), "make -C tests/native (built by __graft_entry__.build)"
    job, out = tmp_path / "job.bin", tmp_path / "out.bin"
    fb = frames[0].nbytes
    with open(job, "wb") as f:
        f.write(b"AQZJ" + struct.pack("<I", len(dims)))
        for d in dims:
            f.write(struct.pack("<iIII", *d))
        f.write(struct.pack("<iiIIQQ", dtype, method, batch, slots, len(frames), fb))
        f.write(np.ascontiguousarray(frames).tobytes())
    r = subprocess.run([exe, str(job), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    log = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert log[-1]["summary"] and log[-1]["ok"]
    got = {}
    b = out.read_bytes()
    assert b[:4] == b"AQZO"
    (nl,), o = struct.unpack_from("<I", b, 4), 8
    for l in range(nl):
        n, lb, nc = struct.unpack_from("<QQI", b, o)
        o += 20
        for _ in range(n):
            (layer,) = struct.unpack_from("<Q", b, o)
            o += 8
            got[(l, layer)] = (np.frombuffer(b, np.uint8, lb, o),
                               np.frombuffer(b, np.uint8, nc, o + lb))
            o += lb + nc
    return log[:-1], got


@pytest.mark.parametrize("case", ["banded-3d", "layers-2d-ragged"])
def test_binding_handoff_replay(gpu, tmp_path, case):
    """The reference-side binding's consumer path, replayed natively: frames
    batched into pinned double buffers, asynchronous appends refilled after
    aqz_stage_wait_consumed, every complete band / layer copied D2H into a
    2-slot host ring and installed when its ticket completes.  Commits are
    contiguous and in frame order per level (Array::write_frame's order,
    array.cpp:196-219), only the partial last unit is unflushed, and every
    installed layer equals the oracle's (MultiscaleArray::write_frame,
    multiscale.array.cpp:57-74, 291-325)."""
    if case == "banded-3d":
        dims = [(TIME, 0, 1, 1), (SPACE, 64, 16, 1), (SPACE, 256, 64, 1), (SPACE, 256, 64, 1)]
        frames = synthetic_frames(U16, 2 * 64 + 24, 256, 256, 61)  # 2 volumes + a partial
        batch = 8
    else:
        dims = [(TIME, 0, 4, 1), (SPACE, 300, 64, 1), (SPACE, 260, 64, 1)]
        frames = synthetic_frames(U16, 4 * 9 + 3, 300, 260, 62)  # ragged last layer
        batch = 5
    exp, fw, _ = expected_stage_layers(dims, U16, MEAN, frames)
    log, got = _run_replay(tmp_path, dims, U16, MEAN, frames, batch, 2)
    per = {}
    for e in log:
        prev = per.setdefault(e["level"], [])
        assert e["first"] == sum(x["frames"] for x in prev), e  # contiguous, in order
        prev.append(e)
    for l, commits in per.items():
        assert sum(c["frames"] for c in commits) == fw[l]
        assert all(c["flush"] for c in commits[:-1])
    if case == "banded-3d":
        assert len(per[0]) > 2 * 4  # bands, not layers
    assert set(got) == set(exp)
    for key, (buf, flags) in exp.items():
        assert_same_pixels(got[key][0].copy(), buf, U16, f"L{key[0]} layer {key[1]}")
        assert np.array_equal(got[key][1], flags), key
