"""GPU: a stage created with aqz_stage_options.level0_split_on_host.

The device runs the pyramid and the split of levels >= 1 only (no level-0
ring in HBM); level 0 is tile-split on the host from the frames the caller
holds (aqz_stage_split_level0_host, the loop of array.cpp:537-619).  Every
level's chunk layers -- level 0 from the host split, levels >= 1 handed off
by D2H -- equal the oracle's (MultiscaleArray::write_frame,
multiscale.array.cpp:57-74, 291-325)."""
import numpy as np
import pytest

from helpers import assert_same_pixels, expected_stage_layers
from oracle_bindings import F32, MEAN, MAX, SPACE, TIME, U8, U16, synthetic_frames

pytestmark = pytest.mark.gpu

CASES = {
    # C2's geometry at a quarter of the size: 512^2 u16, 128^2 chunks, 4 levels
    "c2-small": ([(TIME, 0, 8, 1), (SPACE, 512, 128, 2), (SPACE, 512, 128, 2)], U16, MEAN, 48, 16),
    # ragged tiles at every level, u8, max
    "ragged-u8": ([(TIME, 0, 4, 1), (SPACE, 300, 64, 1), (SPACE, 270, 48, 1)], U8, MAX, 24, 8),
    # 2x2x2: z halves at level 1 (z pairs on the device), f32
    "3d-f32": ([(TIME, 0, 1, 1), (SPACE, 16, 8, 1), (SPACE, 128, 64, 1), (SPACE, 128, 64, 1)],
               F32, MEAN, 48, 16),
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("pinned", [True, False])
def test_host_split_stage_matches_oracle(gpu, case, pinned):
    dims, dt, method, n, B = CASES[case]
    h, w = dims[-2][1], dims[-1][1]
    frames = synthetic_frames(dt, n, h, w, 501)
    frames[3] = 0  # chunks without data
    exp, fw, _ = expected_stage_layers(dims, dt, method, frames)
    st = gpu.Stage(dims, dt, method, max_batch_frames=B, level0_split_on_host=True)
    L = st.n_levels()
    lay = [st.layout(l) for l in range(L)]
    fb = frames[0].nbytes
    src = gpu.HostBuffer(n * fb) if pinned else None
    if pinned:
        src.array[...] = frames.reshape(-1).view(np.uint8)
    host = np.ascontiguousarray(frames)
    F0 = lay[0]["frames_per_layer"]
    lb = [x["bytes_per_chunk"] * x["chunks_per_layer"] for x in lay]
    got = {}
    handed = [0] * L
    for b0 in range(0, n, B):
        if pinned:
            ptr = src.ptr + b0 * fb
            st.append_ptr(ptr, B, gpu.MEM_HOST_PINNED)
        else:
            ptr = host.ctypes.data + b0 * fb
            st.append(host[b0:b0 + B])
        # level 0 on the host, layer by layer, while the batch runs
        f = b0
        while f < b0 + B:
            layer = f // F0
            hi = min(b0 + B, (layer + 1) * F0)
            if (0, layer) not in got:
                got[(0, layer)] = (gpu.HostBuffer(lb[0]), gpu.HostBuffer(lay[0]["chunks_per_layer"]))
                got[(0, layer)][1].array[...] = 0
            buf, hd = got[(0, layer)]
            st.split_level0_host(ptr + (f - b0) * fb, hi - f, f, buf.ptr, lb[0], hd.ptr, hd.nbytes)
            f = hi
        for l in range(1, L):
            while st.frames_written(l) >= (handed[l] + 1) * lay[l]["frames_per_layer"]:
                buf = gpu.HostBuffer(lb[l])
                hd = gpu.HostBuffer(lay[l]["chunks_per_layer"])
                st.copy_layer_async(l, handed[l], buf.ptr, lb[l], hd.ptr, hd.nbytes)
                got[(l, handed[l])] = (buf, hd)
                handed[l] += 1
    st.wait_copies()
    # level 0 has no device layer: every level-0 hand-off call is refused
    for call in (lambda: st.copy_layer_async(0, 0, 0, 0),
                 lambda: st.compress_layer(0, 0, codec=1, clevel=1, shuffle=1)):
        with pytest.raises(gpu.AqzError) as e:
            call()
        assert e.value.status == 1
    full = {k for k in exp if k[0] == 0 or k[1] < handed[k[0]]}
    full = {(l, j) for (l, j) in full if (j + 1) * lay[l]["frames_per_layer"] <= fw[l]}
    assert full and all(k in got for k in full)
    for key in sorted(full):
        buf, hd = got[key]
        layer, flags = exp[key]
        assert_same_pixels(buf.array.copy(), layer, dt, f"{case} level {key[0]} layer {key[1]}")
        assert np.array_equal(hd.array, flags), key
    st.close()


def test_host_split_stage_memory_and_refusals(gpu):
    """No level-0 ring: the estimate and the live device bytes drop by it;
    an XY-transposed storage order is refused (status 9)."""
    dims = [(TIME, 0, 8, 1), (SPACE, 512, 128, 2), (SPACE, 512, 128, 2)]
    est = [gpu.estimate_memory(dims, U16, MEAN, max_batch_frames=16, level0_split_on_host=h)
           for h in (False, True)]
    assert est[1]["device_bytes"] < est[0]["device_bytes"]
    a = gpu.Stage(dims, U16, MEAN, max_batch_frames=16)
    b = gpu.Stage(dims, U16, MEAN, max_batch_frames=16, level0_split_on_host=True)
    ring0 = a.layout(0)["chunk_pitch"] * a.layout(0)["chunks_per_layer"] * a.layout(0)["layer_slots"]
    da, db = a.memory_usage()["device_bytes"], b.memory_usage()["device_bytes"]
    assert da - db >= ring0
    assert db <= est[1]["device_bytes"]
    # frames of two chunk layers in one call are refused (they would land on
    # the same chunks)
    fr = gpu.HostBuffer(16 * 512 * 512 * 2)
    lb = b.layout(0)["bytes_per_chunk"] * b.layout(0)["chunks_per_layer"]
    dst, hd = gpu.HostBuffer(lb), gpu.HostBuffer(b.layout(0)["chunks_per_layer"])
    with pytest.raises(gpu.AqzError) as e:
        b.split_level0_host(fr.ptr, 2, 7, dst.ptr, lb, hd.ptr, hd.nbytes)
    assert e.value.status == 1
    b.split_level0_host(fr.ptr, 8, 8, dst.ptr, lb, hd.ptr, hd.nbytes)
    a.close()
    b.close()
    with pytest.raises(gpu.AqzError) as e:
        gpu.Stage(dims, U16, MEAN, storage_order=[0, 2, 1], level0_split_on_host=True)
    assert e.value.status == 9
