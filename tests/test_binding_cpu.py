"""The binding's host-side helpers on the CPU (integration/aqz_handoff.hh):
AQZ_DEVICE parsing and the z-slab plan, compiled and run natively
(tests/native/binding_host_test.cpp).  The GPU half of the binding runs in
tests/test_gpu_handoff.py."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_binding_host_helpers(tmp_path):
    exe = tmp_path / "binding_host_test"
    r = subprocess.run(["g++", "-std=c++20", "-O1", "-Wall", "-Wextra", "-Werror",
                        "-I", os.path.join(REPO, "include"),
                        "-I", os.path.join(REPO, "integration"),
                        os.path.join(REPO, "tests", "native", "binding_host_test.cpp"),
                        "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr


# BASELINE configs C1-C5 as the binding creates them (64-frame batches)
SHAPES = {
    "c1": ([(2, 0, 64, 1), (0, 512, 128, 1), (0, 512, 128, 1)], 1, 1),
    "c2": ([(2, 0, 64, 1), (0, 2048, 256, 1), (0, 2048, 256, 1)], 1, 1),
    "c3": ([(2, 0, 32, 1), (0, 4096, 128, 1), (0, 4096, 128, 1)], 0, 1),
    "c4": ([(2, 0, 1, 1), (0, 256, 64, 1), (0, 2048, 256, 1), (0, 2048, 256, 1)], 1, 4),
    "c5": ([(2, 0, 4, 1), (0, 8192, 128, 1), (0, 8192, 128, 1)], 8, 1),
}
CODECS = [(0, 0, 0), (1, 5, 1), (2, 5, 2), (3, 1, 0)]


def _handoff_account(dims, dtype, codec, batch, slots, stages, max_batch, layer_slots):
    """The binding's memory, computed independently of estimate_memory:
    Handoff's buffers (aqz_handoff.hh: a batch double buffer per stage;
    per level host_slots unit buffers of the codec's capacity -- the whole
    compressed layer, else a dim-1 band or a layer of raw chunks -- with
    their has_data bytes) and each stage's estimate; per compressed level
    and ring slot the device frames and offsets and their pinned read-back,
    plus the codec scratch."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))
    import aqz
    bpp = {0: 1, 1: 2, 8: 4}[dtype]
    st = aqz.estimate_memory(dims, dtype, 1, max_batch_frames=max_batch,
                             layer_slots=layer_slots, placement_tries=2)
    fb = dims[-1][1] * dims[-2][1] * bpp
    host = stages * (2 * batch * fb + st["pinned_bytes"])
    dev = stages * st["device_bytes"]
    for ld in aqz.pyramid_levels(dims):
        d = aqz.Dims(ld, dtype)
        bpc, n = d.bytes_per_chunk(), d.number_of_chunks_in_memory()
        F = d.frames_per_chunk_layer()
        banded, _, _, per_band = d.dim1_banding()
        if codec[0] or not banded:
            per_band = n
        cap = aqz.compressor_max_bytes(bpc, n) if codec[0] else bpc * per_band
        host += slots * (cap + per_band)
        if codec[0]:
            ring = max(layer_slots, (max_batch - 1 + F - 1) // F + 1)
            offs = (n + 1) * 8
            dev += stages * (ring * (aqz.compressor_max_bytes(bpc, n) + offs) +
                             aqz.compressor_scratch_bytes(codec, bpc, bpp, n))
            host += stages * ring * offs
    return host, dev


def test_binding_memory_estimate_covers_the_handoff():
    """aqz_binding::estimate_memory (what the binding adds to the reference's
    ZarrStreamSettings_estimate_max_memory_usage, acquire.zarr.cpp:216-314)
    for C1-C5 x every codec covers the hand-off's pinned buffers and every
    stage's pinned and device estimate (run natively: tests/native/
    estimate_host, no GPU); the GPU replay checks it against what a live
    hand-off holds (tests/test_gpu_handoff.py)."""
    exe = os.path.join(REPO, "tests", "native", "estimate_host")
    assert os.path.exists(exe), "make -C tests/native (built by __graft_entry__.build)"
    jobs, want = [], []
    for name, (dims, dtype, stages) in SHAPES.items():
        for codec in CODECS:
            args = [len(dims)] + [x for d in dims for x in d] + \
                   [dtype, 64, 3, *codec, stages, 64, 2, 2]
            jobs.append(" ".join(map(str, args)))
            want.append((name, codec, _handoff_account(dims, dtype, codec, 64, 3, stages, 64, 2)))
    env = dict(os.environ)
    env.pop("AQZ_ZSTD_HOST", None)
    r = subprocess.run([exe], input="\n".join(jobs) + "\n", capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    got = [tuple(map(int, l.split())) for l in r.stdout.split("\n") if l.strip()]
    assert len(got) == len(want), r.stdout
    for (name, codec, (h, d)), (eh, ed) in zip(want, got):
        assert eh >= h and ed >= d, (name, codec, eh, h, ed, d)
        assert eh <= 1.01 * h and ed <= 1.01 * d, (name, codec, eh, h, ed, d)
