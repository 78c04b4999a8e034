"""bench.py's link to the committed profiles (no GPU): the device-code hash
of a library (its .hip_fatbin section) and pmc_traffic's choice of summary
-- the same library build first, else a build with the same device code,
else the closest kernel time."""
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

LIB = os.path.join(REPO, "acquire-zarr_amd", "libaqz_gpu.so")


def test_device_code_sha256_reads_the_fatbin_section(tmp_path):
    h = bench.device_code_sha256(LIB)
    assert h and len(h) == 64
    # not the whole file's hash, and stable
    assert h != hashlib.sha256(open(LIB, "rb").read()).hexdigest()
    assert bench.device_code_sha256(LIB) == h
    # a host-only change (bytes appended outside every section) keeps it
    other = tmp_path / "lib.so"
    other.write_bytes(open(LIB, "rb").read() + b"host-only")
    assert bench.device_code_sha256(str(other)) == h
    bad = tmp_path / "x.so"
    bad.write_bytes(b"not an elf")
    assert bench.device_code_sha256(str(bad)) is None
    assert bench.device_code_sha256(str(tmp_path / "missing.so")) is None


def test_pmc_traffic_prefers_same_build_then_same_device_code(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    base = {"config": "c2", "kernel": "k<1>", "ring_allocation": "arena",
            "frames_per_launch": 512}

    def put(name, **kw):
        d = dict(base, **kw)
        (prof / f"{name}_c2_pmc.json").write_text(json.dumps(d))

    put("r90", lib_sha256="aaa", device_code_sha256="D1", traffic_bytes_per_launch=100,
        avg_duration_ns=1.0e6)
    put("r91", lib_sha256="bbb", device_code_sha256="D2", traffic_bytes_per_launch=200,
        avg_duration_ns=2.0e6)
    put("r92", lib_sha256="ccc", device_code_sha256="D1", traffic_bytes_per_launch=300,
        avg_duration_ns=3.0e6)
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    t = lambda **kw: bench.pmc_traffic("c2", False, "k<1>", 512, "arena", **kw)  # noqa: E731
    assert t(run_ms=2.9, lib_sha="bbb")[0] == 200                  # same build
    assert t(run_ms=2.9, lib_sha="zzz", dev_sha="D1")[0] == 300    # same device code, closest
    assert t(run_ms=1.1, lib_sha="zzz", dev_sha="D1")[0] == 100
    assert t(run_ms=2.1, lib_sha="zzz", dev_sha="D9")[0] == 200    # closest of all
    assert bench.pmc_traffic("c2", False, "k<1>", 256, "arena", run_ms=0.5)[0] == 50  # scaled
    assert bench.pmc_traffic("c3", False, "k<1>", 512, "arena")[0] is None
