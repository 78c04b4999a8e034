"""The drop-in boundary, pinned by the compiler (CPU only).

* tests/abi/pin_zarr_types.c includes the reference's public headers
  (include/acquire.zarr.h, zarr.types.h) next to include/aqz_gpu.h and
  _Static_asserts that every AQZ_STATUS_* / AQZ_DTYPE_* / AQZ_DIM_* /
  AQZ_METHOD_* / AQZ_CODEC_* value equals its Zarr* enumerator, and that
  ZarrStreamSettings / ZarrArraySettings / ZarrDimensionProperties keep the
  layout SURVEY.md 8(b) measured (the drop-in changes none of them).
* integration/multiscale.array.gpu.cpp -- the GpuArray / GpuMultiscaleArray
  binding INTEGRATION.md describes -- compiles (-fsyntax-only, -Werror)
  against the reference's own src/streaming headers.
* The drop-in header carries no bench/tuning entry points; those live in
  include/aqz_gpu_bench.h.
"""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
needs_ref = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "include")),
                               reason="reference headers not present (GPU box)")


@needs_ref
def test_enum_values_and_struct_layouts_pinned():
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-fsyntax-only",
                        "-I", os.path.join(REF, "include"), "-I", os.path.join(REPO, "include"),
                        os.path.join(REPO, "tests", "abi", "pin_zarr_types.c")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@needs_ref
def test_pin_detects_a_wrong_value():
    """The pin is live: a header whose value disagrees fails to compile."""
    bad = open(os.path.join(REPO, "include", "aqz_gpu.h")).read().replace(
        "#define AQZ_STATUS_WRITE_OUT_OF_BOUNDS 12", "#define AQZ_STATUS_WRITE_OUT_OF_BOUNDS 11")
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "aqz_gpu.h"), "w").write(bad)
        open(os.path.join(d, "aqz_gpu_bench.h"), "w").write(
            open(os.path.join(REPO, "include", "aqz_gpu_bench.h")).read())
        r = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-I", os.path.join(REF, "include"),
                            "-I", d, os.path.join(REPO, "tests", "abi", "pin_zarr_types.c")],
                           capture_output=True, text=True)
    assert r.returncode != 0 and "AQZ_STATUS_WRITE_OUT_OF_BOUNDS" in r.stderr


@needs_ref
def test_integration_binding_compiles_against_reference_headers():
    nl = os.path.join(REPO, "oracle", "_ref", "include", "nlohmann", "json.hpp")
    if not os.path.exists(nl):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"),
                        "_ref/include/nlohmann/json.hpp"], check=True,
                       stdout=subprocess.DEVNULL)
    streaming = os.path.join(REF, "src", "streaming")
    r = subprocess.run(["g++", "-std=c++20", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                        "-I", os.path.join(REPO, "include"),
                        "-isystem", os.path.join(REPO, "oracle", "_ref", "include"),
                        "-isystem", os.path.join(REF, "include"),
                        "-isystem", streaming,
                        "-isystem", os.path.join(REF, "src", "logger"),
                        "-idirafter", "/opt/conda/include",
                        os.path.join(REPO, "integration", "multiscale.array.gpu.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]


def test_drop_in_header_has_no_bench_entry_points():
    text = open(os.path.join(REPO, "include", "aqz_gpu.h")).read()
    for word in ("force_levels", "skip_level0_split", "blocks_per_cu", "set_tuning",
                 "kernel_timing", "timing_mark", "dominant_kernel"):
        assert word not in text, word
    bench = open(os.path.join(REPO, "include", "aqz_gpu_bench.h")).read()
    for word in ("force_levels", "skip_level0_split", "aqz_stage_set_tuning",
                 "aqz_stage_timing_mark", "aqz_stage_dominant_kernel"):
        assert word in bench, word
    # both headers compile as C and as C++ on their own
    for lang, std in (("c", "c11"), ("c++", "c++17")):
        r = subprocess.run(["gcc", "-x", lang, f"-std={std}", "-Wall", "-Werror",
                            "-fsyntax-only", "-I", os.path.join(REPO, "include"), "-"],
                           input='#include "aqz_gpu_bench.h"\n', capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
