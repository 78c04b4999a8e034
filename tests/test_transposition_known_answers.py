"""storage_dimension_order pinned to the reference's own known answers
(python/tests/test_dimension_transposition.py, restated as data):

* test_dimension_transposition (:55-156): 5-D t/c/z/y/x dims (t 2 chunk 1,
  c 3, z 4, y 16 chunk 8, x 24 chunk 8), frames np.full(frame, i) in
  acquisition order; stored[..., 0, 0] must equal
  arange(n).reshape(acquisition append shape) transposed by the storage
  permutation -- identity, explicit identity, z<->c, and z<->c with an
  unbounded t (array size 0, 5 time points);
* test_swap_xy (:185-206): t/y/x with storage order t/x/y, one frame whose
  row y holds the value y; the stored plane is x_size rows of
  range(y_size).

The CPU test runs the oracle (the C restatement's tile split behind the
compiled reference's transpose_frame_id when oracle/_ref is built); the GPU
test runs the stage.  `array.cpp` (transpose_frame, :488-504) does not
build here, so these known answers are what pins the XY order (SURVEY 8a
a13/f4) to the reference."""
import numpy as np
import pytest

from helpers import assemble_layers, expected_stage_layers
from oracle_bindings import CHANNEL, MEAN, SPACE, TIME, U8, U16, OracleDims, ref_available

DIMS = {"t": (TIME, 2, 1, 1), "c": (CHANNEL, 3, 1, 1), "z": (SPACE, 4, 1, 1),
        "y": (SPACE, 16, 8, 1), "x": (SPACE, 24, 8, 1)}
CASES = {
    "identity": ("tczyx", None, None),
    "identity-explicit": ("tczyx", "tczyx", None),
    "zc-swap": ("tzcyx", "tczyx", None),
    "zc-swap-unbounded": ("tzcyx", "tczyx", 5),
}


def _case(name):
    inp, out, append = CASES[name]
    out = out or inp
    acq = [DIMS[d] for d in inp]
    if append is not None:
        acq[0] = (acq[0][0], 0, acq[0][2], acq[0][3])
    perm = [inp.index(d) for d in out]
    size = {d: (append if (i == 0 and append is not None) else DIMS[d][1])
            for i, d in enumerate(inp)}
    in_shape = [size[d] for d in inp]
    n = int(np.prod(in_shape[:-2]))
    frames = np.stack([np.full(in_shape[-2:], v, dtype=np.uint8) for v in range(n)])
    expect = np.arange(n, dtype=np.uint8).reshape(in_shape[:-2])
    if out != inp:
        expect = np.transpose(expect, [inp.index(d) for d in out[:-2]])
    return acq, perm, frames, expect


def _stored_frame_values(layers0, sdims):
    return assemble_layers(layers0, sdims, U8)[..., 0, 0]


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_transposition_known_answers(name):
    acq, perm, frames, expect = _case(name)
    sdims = [acq[i] for i in perm]
    if ref_available():
        fid = OracleDims(acq, U8, use_ref=True, order=perm).transpose_frame_id
    else:
        import aqz
        fid = aqz.Dims(acq, U8, storage_order=perm).transpose_frame_id
    exp, fw, _ = expected_stage_layers(sdims, U8, MEAN, frames, storage_fid=fid)
    got = _stored_frame_values({k: v[0] for (l, k), v in exp.items() if l == 0}, sdims)
    assert np.array_equal(got, expect)


def test_oracle_swap_xy_known_answer():
    y, x = DIMS["y"][1], DIMS["x"][1]
    frame = np.broadcast_to(np.arange(y, dtype=np.uint8)[:, None], (y, x))
    sdims = [DIMS["t"], DIMS["x"], DIMS["y"]]
    exp, _, _ = expected_stage_layers(sdims, U8, MEAN, np.ascontiguousarray(frame.T)[None])
    got = assemble_layers({k: v[0] for (l, k), v in exp.items() if l == 0}, sdims, U8)
    assert np.array_equal(got[0], np.array([list(range(y))] * x, dtype=np.uint8))


def _stage_level0(gpu, acq, perm, frames, dtype, batch=5):
    st = gpu.Stage(acq, dtype, MEAN, storage_order=perm if perm != list(range(len(acq)))
                   else None, max_batch_frames=batch, layer_slots=8)
    for b0 in range(0, len(frames), batch):
        st.append(np.ascontiguousarray(frames[b0:b0 + batch]))
    st.finalize()
    F = st.layout(0)["frames_per_layer"]
    n_layers = -(-st.frames_written(0) // F)
    layers = {k: st.copy_layer(0, k)[0].tobytes() for k in range(n_layers)}
    st.close()
    return layers


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_stage_transposition_known_answers(gpu, name):
    acq, perm, frames, expect = _case(name)
    layers = _stage_level0(gpu, acq, perm, frames, U8)
    got = _stored_frame_values(layers, [acq[i] for i in perm])
    assert np.array_equal(got, expect)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(16, 24, 8, U8), (1000, 1088, 128, U16), (130, 77, 16, U16)],
                         ids=["reference", "fused-strip", "ragged"])
def test_stage_swap_xy_known_answer(gpu, shape):
    """The reference's frame (row y = y) at its own size, and at sizes that
    take the fused strip kernel's XY loads and ragged transpose tiles."""
    y, x, c, dt = shape
    npdt = np.uint8 if dt == U8 else np.uint16
    frame = np.broadcast_to(np.arange(y, dtype=npdt)[:, None], (y, x))
    acq = [(TIME, 2, 1, 1), (SPACE, y, c, 1), (SPACE, x, c, 1)]
    layers = _stage_level0(gpu, acq, [0, 2, 1], np.ascontiguousarray(frame)[None], dt)
    got = assemble_layers(layers, [acq[0], acq[2], acq[1]], dt)
    assert got.shape[1:] == (x, y)
    assert np.array_equal(got[0], np.array([list(range(y))] * x, dtype=npdt))
