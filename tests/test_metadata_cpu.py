"""OME downsampling metadata, byte for byte.

MultiscaleArray embeds Downsampler::downsampling_method() as
multiscales[0].type and get_metadata() as multiscales[0].metadata in
zarr.json (multiscale.array.cpp:268-271).  The stage's strings
(aqz_downsampling_method_name / aqz_downsampling_metadata_json, the same
code aqz_downsampler_* returns) must equal the compiled reference's
get_metadata().dump() (downsampler.cpp:422-485).  tests/golden/metadata.json
holds the reference's strings (tests/golden/make_golden.py) so the check
also runs where the reference is absent.  The dump was produced with the
image's nlohmann 3.1.1; compact dump() output (sorted object keys, no
spaces) is the same in the nlohmann the reference pins."""
import ctypes as C
import json
import os

import pytest

import aqz
import oracle_bindings as ob

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "metadata.json")


def golden():
    return json.load(open(GOLDEN))


@pytest.mark.parametrize("method", range(4))
def test_metadata_matches_golden(method):
    g = golden()[str(method)]
    assert aqz.downsampling_method_name(method) == g["method_name"]
    assert aqz.downsampling_metadata_json(method) == g["metadata"]


@pytest.mark.skipif(not ob.ref_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("method", range(4))
def test_metadata_matches_compiled_reference(method):
    R = ob.ref()
    R.ref_ds_metadata.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
    R.ref_ds_metadata.restype = C.c_size_t
    R.ref_ds_method_name.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
    R.ref_ds_method_name.restype = C.c_size_t
    ds = ob.OracleDownsampler([(ob.TIME, 0, 5, 1), (ob.SPACE, 10, 5, 1), (ob.SPACE, 10, 5, 1)],
                              ob.U16, method, 0, use_ref=True)
    buf = C.create_string_buffer(4096)
    n = R.ref_ds_metadata(ds.h, buf, 4096)
    assert aqz.downsampling_metadata_json(method).encode() == buf.value and n == len(buf.value)
    name = C.create_string_buffer(64)
    R.ref_ds_method_name(ds.h, name, 64)
    assert aqz.downsampling_method_name(method).encode() == name.value


def test_metadata_invalid_method_and_small_buffer():
    with pytest.raises(aqz.AqzError) as e:
        aqz.downsampling_metadata_json(4)
    assert e.value.status == 1
    assert aqz.downsampling_method_name(-1) == ""
    n = C.c_size_t(0)
    assert aqz.lib().aqz_downsampling_metadata_json(1, None, 0, C.byref(n)) == 0
    buf = C.create_string_buffer(int(n.value))  # no room for the NUL
    assert aqz.lib().aqz_downsampling_metadata_json(1, buf, n.value, C.byref(n)) == 2
