"""End to end through the C ABI, from a host frame buffer to shard files
(acquire-zarr_amd/examples/stream_to_filesystem, native C++): frames ->
H2D -> stage -> [device blosc1-lz4] -> D2H -> Zarr v3 shard files with the
index table + CRC-32C at the end (shard.cpp:145-166), at the reference's
shard paths <level>/c/<append shard>/<y shard>/<x shard> (array.cpp:130-135,
sink.cpp:47-100).  Every chunk read back from the files -- raw or decoded --
equals the oracle's chunk of MultiscaleArray::write_frame for the same
frames; chunks without data and the zero-filled partial last layer follow
the reference (skip sentinel, lazily zeroed chunks)."""
import os
import struct
import subprocess

import numpy as np
import pytest

from codec_helpers import blosc_zstd_decode, crc32c, libzstd, oracle_decode, zstd_decode
from helpers import expected_stage_layers
from oracle_bindings import MEAN, SPACE, TIME, U16, OracleDims, OracleDownsampler, \
    synthetic_frames

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "acquire-zarr_amd", "examples", "stream_to_filesystem")
# the example's "c1" preset: BASELINE configs[0], u16 512x512, 3 levels
DIMS = [(TIME, 0, 64, 1), (SPACE, 512, 128, 2), (SPACE, 512, 128, 2)]
UNWRITTEN = (1 << 64) - 1


def read_shard(path, cps):
    blob = open(path, "rb").read()
    tbl = blob[len(blob) - 16 * cps - 4:]
    body, crc = tbl[:-4], struct.unpack("<I", tbl[-4:])[0]
    assert crc32c(body) == crc, f"shard index checksum of {path}"
    pairs = [struct.unpack("<QQ", body[16 * i:16 * i + 16]) for i in range(cps)]
    return blob, pairs


def shards_along(level_dims):
    out = []
    for _, size, chunk, shard in level_dims[1:]:
        chunks = -(-size // chunk)
        out.append(-(-chunks // max(1, shard)))
    return out


@pytest.mark.parametrize("codec,shuffle,source", [("lz4", 2, "pinned"), ("lz4", 1, "pageable"),
                                                  ("raw", 0, "pinned"),
                                                  ("blosc-zstd", 1, "pinned"),
                                                  ("zstd", 0, "pinned")])
def test_stream_to_filesystem_shards(gpu, tmp_path, codec, shuffle, source):
    assert os.path.exists(EXE), "build acquire-zarr_amd (make) first"
    if "zstd" in codec and libzstd() is None:
        pytest.skip("libzstd.so.1 absent")
    n, seed = 100, 31  # one full t-chunk layer + a partial one
    out = tmp_path / "store"
    r = subprocess.run([EXE, str(out), "--config", "c1", "--frames", str(n), "--ring", str(n),
                        "--codec", codec, "--shuffle", str(shuffle), "--source", source,
                        "--seed", str(seed), "--writers", "4"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert '"metric"' in r.stdout

    frames = synthetic_frames(U16, n, 512, 512, seed)
    exp, fw, _ = expected_stage_layers(DIMS, U16, MEAN, frames)
    ods = OracleDownsampler(DIMS, U16, MEAN, 0)
    checked = 0
    for level in range(ods.n_levels()):
        ld = ods.level_dims(level)
        od = OracleDims(ld, U16)
        cim, bpc = od.number_of_chunks_in_memory(), od.bytes_per_chunk()
        # ArrayDimensions::chunks_per_shard / chunk_layers_per_shard
        # (array.dimensions.cpp:172, 388-391)
        cps = int(np.prod([d[3] for d in ld]))
        lps = ld[0][3]
        along = shards_along(ld)
        layers = sorted(k[1] for k in exp if k[0] == level)
        assert layers, level
        for row in sorted({lay // lps for lay in layers}):
            want = {}
            for cl in range(lps):
                layer = row * lps + cl
                if (level, layer) not in exp:
                    continue
                buf, flags = exp[(level, layer)]
                for c in range(cim):
                    idx = cl * cim + c
                    key = (od.shard_index_for_chunk(idx), od.shard_internal_index(idx))
                    want[key] = buf[c * bpc:(c + 1) * bpc].tobytes() if flags[c] else None
            for s in range(int(np.prod(along))):
                co = np.unravel_index(s, along)
                path = os.path.join(out, str(level), "c", str(row), *map(str, co))
                blob, pairs = read_shard(path, cps)
                for i, (off, ext) in enumerate(pairs):
                    w = want.get((s, i))
                    if w is None:
                        assert off == UNWRITTEN and ext == UNWRITTEN, (level, row, s, i)
                        continue
                    got = blob[off:off + ext]
                    if codec == "lz4":
                        got = oracle_decode(got)
                    elif codec == "blosc-zstd":
                        got = blosc_zstd_decode(got)
                    elif codec == "zstd":
                        got = zstd_decode(got, bpc)
                    assert got == w, (level, row, s, i)
                    checked += 1
    assert checked > 0
