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
