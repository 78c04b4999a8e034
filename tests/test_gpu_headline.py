"""GPU parity of exactly what bench.py times.

* C2 as benched: u16 2048x2048, 256-px chunks, t-chunk 64, force_levels=5
  (the BASELINE "5-level @ 256-px chunks" geometry; the reference rule
  stops at 4 levels, downsampler.cpp:512-541), the bench's launch size
  and chunk-layer ring, from a device-resident ring of frames.  Pixels of every
  level come from the oracle run at 128-px chunks (5 levels by the
  reference rule, the same pixels -- level values do not depend on the
  chunk size) tiled at the forced 256-px level dims.
* c2-ref4: the same frames under the reference level rule (4 levels).
* C4 as stated in BASELINE configs[3]: u16 2048x2048x256 planes, z-chunk 64,
  128-plane launches (fused 2x2x2 kernel); then the same volume split into
  4 z slabs (what --gpus 4 runs: aqz.dist.z_slab(256, 4, r, 4)), one stage
  per slab with first_frame = the slab's first plane; the slabs' chunk
  layers assemble, with no exchange, into the single-volume result.

Reference: downsampler.cpp:306-414, 494-597; array.cpp:507-622.
"""
import numpy as np
import pytest

import bench
from helpers import assert_same_pixels, expected_stage_layers
from oracle_bindings import MEAN, SPACE, U16, synthetic_frames

pytestmark = pytest.mark.gpu


def distinct_frames(n, h, w, seed, base=8):
    """n distinct u16 frames: `base` splitmix frames, frame i XOR-ed with a
    per-frame constant (cheap at GiB scale, and no two frames equal)."""
    b = synthetic_frames(U16, min(n, base), h, w, seed)
    out = np.empty((n, h, w), np.uint16)
    for i in range(n):
        np.bitwise_xor(b[i % len(b)], np.uint16((i * 40503 + 1) & 0xFFFF), out=out[i])
    return out


def _device_ring(frames):
    import torch
    t = torch.from_numpy(frames.view(np.int16)).cuda()
    torch.cuda.synchronize()
    return t


def _check_layer(st, l, layer, exp):
    buf, flags = exp.pop((l, layer))
    got, gflags = st.copy_layer(l, layer)
    assert_same_pixels(got, buf, U16, f"L{l} layer{layer}")
    assert np.array_equal(gflags, flags), f"has_data L{l} layer{layer}"


@pytest.mark.parametrize("cfg", ["c2", "c2-ref4", "c2-xy"])
def test_bench_c2_configuration_exact(gpu, cfg):
    """The bench's C2 stages, placement search included, oracle-exact;
    c2-xy is `bench.py --xy` (XY-transposed storage order, the transpose
    fused into the strip kernel's loads)."""
    xy = cfg == "c2-xy"
    c = bench.CONFIGS["c2" if xy else cfg]
    dims, B = c["dims"], c["batch"]
    h, w = dims[-2][1], dims[-1][1]
    slots = bench.layer_slots_for(c, B)
    kw = dict(force_levels=c["force_levels"], max_batch_frames=B, layer_slots=slots,
              **bench.PLACEMENT)
    if xy:
        assert h == w  # storage dims equal acquisition dims
        kw["storage_order"] = [0, 2, 1]
    est = gpu.estimate_memory(dims, U16, MEAN, **kw)
    st = gpu.Stage(dims, U16, MEAN, **kw)
    L = st.n_levels()
    assert L == (4 if cfg == "c2-ref4" else 5)
    # the bench's placement search ran (the arena against the probe of its
    # memory); its creation peak is within the bench estimate, and the stage
    # keeps one ring set afterwards
    pl = st.placement()
    assert 1 <= len(pl["candidates_ms"]) <= bench.PLACEMENT["placement_tries"]
    assert pl["candidates_ms"][pl["kept"]] == min(pl["candidates_ms"])
    assert 0 < pl["kept_ms_final"] and pl["mode"] == 3 and pl["probe_bus_gbs"] > 0
    assert pl["accepted"] or len(pl["candidates_ms"]) == bench.PLACEMENT["placement_tries"]
    assert pl["peak_device_bytes"] <= est["device_bytes"]
    assert st.memory_usage()["device_bytes"] <= gpu.estimate_memory(
        dims, U16, MEAN, force_levels=c["force_levels"], max_batch_frames=B,
        layer_slots=slots, storage_order=kw.get("storage_order"))["device_bytes"]
    ldims = [st.level_dims(l) for l in range(L)]
    assert [d[-1][1] for d in ldims] == [2048, 1024, 512, 256, 128][:L]
    assert all(d[-1][2] == 256 and d[-2][2] == 256 for d in ldims)
    if cfg == "c2":
        assert st.dominant_kernel() == "fused_pyramid_strip"
    if xy:
        assert st.dominant_kernel() == "fused_pyramid_strip (XY load)"
    # oracle pixels: the reference rule at 128-px chunks gives the same
    # 5 levels (c2); c2-ref4 is the reference configuration itself
    odims = list(dims)
    if c["force_levels"]:  # c2, c2-xy
        odims[-1] = (SPACE, w, 128, 1)
        odims[-2] = (SPACE, h, 128, 1)
    # one full launch and a half one: more frames than the ring's slots hold
    # (9 layers of 64 at B = 512), so every slot is reused once
    n = B + B // 2
    frames = distinct_frames(n, h, w, 7 + L)
    stored = np.ascontiguousarray(frames.transpose(0, 2, 1)) if xy else frames
    exp, fw, _ = expected_stage_layers(odims, U16, MEAN, stored, level_dims=ldims)
    del stored
    assert len(fw) == L
    ring = _device_ring(frames)
    F = [st.layout(l)["frames_per_layer"] for l in range(L)]
    done = [0] * L
    for s in range(0, n, B):
        st.append_ptr(ring.data_ptr() + s * h * w * 2, min(B, n - s))
        st.synchronize()
        # check every layer completed by this launch before the 3-slot
        # ring reuses its slot
        for l in range(L):
            while (done[l] + 1) * F[l] <= st.frames_written(l):
                _check_layer(st, l, done[l], exp)
                done[l] += 1
    for l in range(L):
        assert st.frames_written(l) == fw[l]
    assert not exp, f"unchecked layers: {sorted(exp)}"
    st.close()


@pytest.fixture(scope="module")
def c4_volume():
    c = bench.CONFIGS["c4"]
    dims = c["dims"]
    Z, h, w = dims[1][1], dims[-2][1], dims[-1][1]
    assert (Z, h, w) == (256, 2048, 2048) and dims[1][2] == 64
    frames = distinct_frames(Z, h, w, 404)
    exp, fw, ldims = expected_stage_layers(dims, U16, MEAN, frames)
    return c, frames, exp, fw, ldims


def test_c4_volume_exact(gpu, c4_volume):
    c, frames, exp, fw, ldims = c4_volume
    dims, B = c["dims"], c["batch"]
    st = gpu.Stage(dims, U16, MEAN, max_batch_frames=B, layer_slots=2)
    assert st.dominant_kernel() == "fused_pyramid_strip3d_pair"
    assert st.n_levels() == 4 == len(ldims)
    assert [st.level_dims(l)[1][1] for l in range(4)] == [256, 128, 64, 64]
    ring = _device_ring(frames)
    fbytes = frames[0].nbytes
    for s in range(len(frames) // B):
        st.append_ptr(ring.data_ptr() + s * B * fbytes, B)
    st.finalize()
    for l in range(4):
        assert st.frames_written(l) == fw[l], (l, st.frames_written(l), fw[l])
    for (l, layer), (buf, flags) in sorted(exp.items()):
        got, gflags = st.copy_layer(l, layer)
        assert_same_pixels(got, buf, U16, f"L{l} layer{layer}")
        assert np.array_equal(gflags, flags), (l, layer)
    st.close()


def test_c4_z_slabs_over_4_stages(gpu, c4_volume):
    """The --gpus 4 decomposition on one device: 4 stages own the z slabs
    [64r, 64r+64) of every volume (z_slab schedule) and get two volumes of a
    stream (the second volume repeats the first's planes); OR-ing their chunk
    layers gives exactly the single-stream layers of both volumes (each slab
    writes only its own chunk regions; the rest stays 0)."""
    import aqz
    from aqz.dist import z_levels, z_slab
    c, frames, exp, fw, ldims = c4_volume
    dims = c["dims"]
    planes = [lv[1][1] for lv in aqz.pyramid_levels(dims)]
    align = 1 << z_levels(planes)
    assert align == 4
    ring = _device_ring(frames)
    fbytes = frames[0].nbytes
    stages = []
    for r in range(4):
        lo, hi = z_slab(planes[0], 4, r, align)
        assert (lo, hi) == (64 * r, 64 * r + 64)
        st = gpu.Stage(dims, U16, MEAN, max_batch_frames=c["batch"], layer_slots=2,
                       z_slab=(lo, hi))
        for vol in range(2):
            st.append_ptr(ring.data_ptr() + lo * fbytes, hi - lo)
        stages.append(st)
    for st in stages:
        st.finalize()
    for l in range(4):  # every stage's frame id is at its slab of volume 3
        assert stages[-1].frames_written(l) == 2 * fw[l] + fw[l] * 3 // 4
    for (l, layer), (buf, flags) in sorted(exp.items()):
        for vol in range(2):
            acc, facc = None, None
            for st in stages:
                got, gflags = st.copy_layer(l, layer + vol)
                acc = got if acc is None else np.bitwise_or(acc, got, out=acc)
                facc = gflags if facc is None else np.maximum(facc, gflags)
            assert_same_pixels(acc, buf, U16, f"slabs L{l} layer{layer + vol}")
            assert np.array_equal(facc, flags), (l, layer + vol)
    for st in stages:
        st.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("extra", [[], ["--config", "c4"],
                                   ["--e2e", "pinned", "--compress", "1"]],
                         ids=["c2", "c4-zslab", "e2e-lz4"])
def test_bench_two_ranks_self_launched(gpu, extra):
    """`bench.py --gpus 2` with no launcher starts 2 ranks itself (both on
    this box's one GPU, gloo for the barrier / max) and reports n_gpus 2:
    the headline line, C4 with each rank on its own z slab, and the
    end-to-end hand-off with device compression."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, AQZ_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2",
                        "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                        "--no-pyramid-only-line", "--no-hbm-probe"] + extra,
                       capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0
    if "--e2e" not in extra:
        # each rank's kernel time, placement and creation cost, gathered
        # into rank 0's line
        pr = d["per_rank"]
        assert [r["rank"] for r in pr] == [0, 1]
        for r in pr:
            assert r["kernel_avg_ms"] > 0 and r["stage_create_s"] > 0
            assert r["peak_device_bytes"] > 0 and len(r["candidates_ms"]) >= 1
            assert 0 < r["elapsed_s"] <= 1.01 * d["ms_per_step"] * d["steps"] / 1e3 + 1e-5


def test_hbm_probe_shapes(gpu):
    """The live streaming probe the bench reports its ceilings from
    (aqz_probe_hbm): every shape runs, reads what it says, and lands in a
    plausible band for one MI355X (0.5-8.5 TB/s of bus); bad shapes are
    refused."""
    for shape, wr in ((gpu.PROBE_READ, 0.0), (gpu.PROBE_COPY, 1.0),
                      (gpu.PROBE_COPY_THIRD, 4 / 3), (gpu.PROBE_READ_THIRD, 1 / 3),
                      (gpu.PROBE_COPY | gpu.PROBE_PLAIN_STORES, 1.0)):
        ms, rd = gpu.probe_hbm(shape, 256 << 20, 5)
        assert 0 < rd <= 256 << 20 and rd > 255 << 20
        bus = rd * (1 + wr) / (ms * 1e-3) / 1e9
        assert 500 < bus < 8500, (shape, bus)
    with pytest.raises(gpu.AqzError):
        gpu.probe_hbm(7, 1 << 20, 1)


def _paced(extra):
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--config", "c3",
                        "--e2e", "pinned"] + extra, capture_output=True, text=True,
                       timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return lines[0]


@pytest.mark.timeout(300)
def test_paced_camera_accounting():
    """bench.py's simulated camera (run_paced): u8 4096x4096 frames land in a
    pinned ring at a fixed rate and are appended in batches of 8 as they
    arrive.  At a rate the stage sustains nothing is dropped and every frame
    is processed; with a ring too small for the rate, frames the camera
    overwrote before the stage read them are counted as drops, and every
    frame is either processed or dropped -- never both, never lost."""
    ok = _paced(["--fps", "200", "--seconds", "1", "--batch", "8"])
    assert ok["frames"] == 200 and ok["drops"] == 0
    assert ok["processed"] == ok["appended"] == ok["stage_frames_written"] == 200
    assert ok["value"] > 150  # sustained fps near the target
    # 10000 fps (160 GB/s of frames) into a 16-frame ring: PCIe cannot keep up
    over = _paced(["--fps", "10000", "--seconds", "0.3", "--batch", "8",
                   "--camera-ring", "16"])
    assert over["drops"] > 0
    assert over["processed"] + over["drops"] == over["frames"] == 3000
    assert over["appended"] == over["processed"] == over["stage_frames_written"]
