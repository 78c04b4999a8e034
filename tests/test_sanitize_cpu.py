"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5
"Race detection / sanitizers": build a -fsanitize=address,undefined host
variant of the CPU restatement and the shim).

tests/sanitize/host_sanitize.cpp is compiled with the product's pure-host
sources (geometry restatement, staging copy pool, host zstd pool + frame
writer) and the CPU oracle, all instrumented, and run; any ASan/UBSan
report aborts it.  tests/sanitize/capi_sanitize.cpp does the same for the host-only entry
points of the C ABI: csrc/aqz_capi.cpp and csrc/aqz_geometry.cpp are
compiled host-side (hipcc --cuda-host-only, the sanitizers on the host
only) and linked ahead of libaqz_gpu.so, so the instrumented definitions
run.  The HIP kernels and the device engine are not host code and GPU
sanitizers are not available on this pool."""
import os
import subprocess

import pytest

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "acquire-zarr_amd", "libaqz_gpu.so")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "acquire-zarr_amd", "csrc")


def test_host_code_clean_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_sanitize")
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=undefined", "-pthread"]
    objs = []
    for src in ("oracle/aqz_oracle.c", "oracle/aqz_codec_oracle.c"):
        o = str(tmp_path / (os.path.basename(src) + ".o"))
        r = subprocess.run(["gcc", "-std=c11", "-ffp-contract=off", *flags, "-c",
                            os.path.join(REPO, src), "-o", o], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        objs.append(o)
    srcs = [os.path.join(REPO, "tests", "sanitize", "host_sanitize.cpp")] + [
        os.path.join(CSRC, f) for f in ("aqz_geometry.cpp", "aqz_copy.cpp", "aqz_hostsplit.cpp",
                                        "aqz_hostzstd.cpp")]
    r = subprocess.run(["g++", "-std=c++20", *flags, "-I", CSRC, "-I",
                        os.path.join(REPO, "oracle"), *srcs, *objs, "-ldl", "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "clean" in r.stdout
    assert "runtime error" not in r.stderr


@pytest.mark.skipif(not os.path.exists(LIB), reason="libaqz_gpu.so not built")
def test_capi_host_entry_points_clean_under_asan_ubsan(tmp_path):
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not present")
    inc = ["-I", os.path.join(REPO, "include"), "-I", CSRC]
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=undefined"]
    common = ["-std=c++20", "-O1", "-g", "-fPIC", "-fno-omit-frame-pointer"]
    objs = []
    for src, lang in ((os.path.join(CSRC, "aqz_capi.cpp"), ["-x", "hip", "--cuda-host-only"]),
                      (os.path.join(CSRC, "aqz_geometry.cpp"), ["-x", "c++"]),
                      (os.path.join(REPO, "tests", "sanitize", "capi_sanitize.cpp"), ["-x", "c++"])):
        o = str(tmp_path / (os.path.basename(src) + ".o"))
        r = subprocess.run([hipcc, *lang, *common, *inc, *san, "-c", src, "-o", o],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-4000:]
        objs.append(o)
    exe = str(tmp_path / "capi_sanitize")
    libdir = os.path.dirname(LIB)
    r = subprocess.run([hipcc, "-fsanitize=address,undefined", "-fno-gpu-sanitize", *objs,
                        "-L", libdir, "-laqz_gpu", "-L/opt/rocm/lib", "-l:libamdhip64.so.7",
                        f"-Wl,-rpath,{libdir}", "-Wl,-rpath,/opt/rocm/lib", "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "clean" in r.stdout
    assert "runtime error" not in r.stderr
