"""The Python mirror's structs (acquire-zarr_amd/aqz/__init__.py, ctypes)
against the C headers they mirror (include/aqz_gpu.h, aqz_gpu_bench.h):
size and every field's offset, from a C program compiled here.  A field
added to a header but not to the mirror (or the reverse) would shift every
field after it and be read as garbage by the tests and the bench."""
import ctypes as C
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acquire-zarr_amd"))

import aqz  # noqa: E402

PAIRS = {
    "aqz_dimension": aqz.Dimension,
    "aqz_array_desc": aqz.ArrayDescC,
    "aqz_stage_options": aqz.StageOptionsC,
    "aqz_stage_bench_options": aqz.StageBenchOptionsC,
    "aqz_placement_report": aqz.PlacementReportC,
    "aqz_memory_usage": aqz.MemoryUsageC,
    "aqz_compression": aqz.CompressionC,
    "aqz_chunk_entry": aqz.ChunkEntryC,
    "aqz_level_layout": aqz.LevelLayoutC,
}


def test_ctypes_mirror_matches_the_headers(tmp_path):
    pairs = PAIRS
    lines = ['#include "aqz_gpu_bench.h"', "#include <stddef.h>", "#include <stdio.h>",
             "int main(void) {"]
    for cname, py in pairs.items():
        lines.append(f'    printf("{cname} size %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'    printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines += ["    return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"),
                        str(src), "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    got = {}
    for line in out.splitlines():
        name, field, val = line.split()
        got[(name, field)] = int(val)
    for cname, py in pairs.items():
        assert got[(cname, "size")] == C.sizeof(py), cname
        for f in py._fields_:
            assert got[(cname, f[0])] == getattr(py, f[0]).offset, (cname, f[0])
