"""The binding harness without a GPU (oracle/_ref/binding_exec, built where
/root/reference exists): the hook declines the array -- make_gpu_multiscale_
array returns nullptr when no device is visible, so the stream keeps the
reference's CPU path (zarr.stream.cpp:1231-1279)
-- and the constructor, asked for a stage anyway, fails loudly instead of
falling back to anything."""
import os
import struct
import subprocess

import numpy as np
import pytest

from oracle_bindings import MEAN, SPACE, TIME, U16

EXE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle", "_ref",
                   "binding_exec")
pytestmark = pytest.mark.skipif(not os.path.exists(EXE), reason="make -C oracle binding")


def _job(tmp_path, batch):
    dims = [(TIME, 0, 4, 2), (SPACE, 64, 32, 1), (SPACE, 64, 32, 1)]
    job = tmp_path / "job.bin"
    with open(job, "wb") as f:
        f.write(b"AQZ2" + struct.pack("<I", len(dims)))
        for d in dims:
            f.write(struct.pack("<iIII", *d))
        f.write(struct.pack("<iiIIiiiiIIIIIQQ", U16, MEAN, batch, 2, 0, 0, 0, 0, 0, 2, 0, 0, 1,
                            8, 64 * 64 * 2))
        f.write(np.zeros((8, 64, 64), np.uint16).tobytes())
    return job


def _run(tmp_path, batch):
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    return subprocess.run([EXE, str(_job(tmp_path, batch)), str(tmp_path / "out.bin")],
                          capture_output=True, text=True, timeout=120, env=env)


def test_hook_declines_without_a_device(tmp_path):
    r = _run(tmp_path, 0)
    assert r.returncode == 1 and "make_gpu_multiscale_array: nullptr" in r.stderr, r.stderr


def test_constructor_fails_loudly_without_a_device(tmp_path):
    r = _run(tmp_path, 4)
    assert r.returncode == 1, r.stderr
    assert "aqz_stage_create failed" in r.stderr or "aqz_device_count" in r.stderr, r.stderr


def test_malformed_job_is_refused(tmp_path):
    bad = tmp_path / "bad.bin"
    bad.write_bytes(b"AQZ9")
    r = subprocess.run([EXE, str(bad), str(tmp_path / "o.bin")], capture_output=True,
                       timeout=60)
    assert r.returncode == 2
