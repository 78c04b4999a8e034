"""GPU tests of the chunk-layer ring placement.

* The creation-time search (aqz_stage_options.placement_tries): the rings as
  created are timed against the stage's algorithmic bytes at the rate of a
  copy-third streaming probe of the same memory; fresh arenas follow only
  while the best is over that expectation, each made while the best is held
  and freed at once when it loses.  Its worst case (every try run) stays
  within aqz_stage_estimate_memory.
* Device memory comes back when a stage with a ring arena is destroyed (the
  arena's 2 MiB pieces are unmapped one by one).
* z slabs whose rings are views into VMM arenas: aqz_stage_import_frames
  reads one stage's arena from another (on a second device when there is
  one, which maps the arena for it: Stage::grant_access).

Reference: downsampler.cpp:306-414; array.cpp:507-622 (the chunk layers);
acquire.zarr.cpp:216-314 (the memory estimate's contract).
"""
import numpy as np
import pytest

from helpers import assert_same_pixels, expected_stage_layers
from oracle_bindings import MEAN, SPACE, TIME, U16, synthetic_frames

pytestmark = pytest.mark.gpu

C2 = [(TIME, 0, 64, 1), (SPACE, 2048, 256, 1), (SPACE, 2048, 256, 1)]


def test_placement_search_reports_its_expectation(gpu):
    """The search on the binding's geometry (64-frame launches; 4 tries
    here, the binding passes 2): candidate 0 is the ring arena, the probe
    ran over its memory, and the search stopped either at a candidate within
    3% of the expectation or after every try."""
    kw = dict(force_levels=5, max_batch_frames=64, layer_slots=2, placement_tries=4)
    est = gpu.estimate_memory(C2, U16, MEAN, **kw)
    st = gpu.Stage(C2, U16, MEAN, **kw)
    pl = st.placement()
    st.close()
    assert pl["mode"] == 3  # ring arenas of 2 MiB pieces
    ms = pl["candidates_ms"]
    assert 1 <= len(ms) <= 4 and pl["kept"] == ms.index(min(ms))
    assert 500 < pl["probe_bus_gbs"] < 8500
    # 64 frames: in + split + the four levels' tiles
    fb = 2048 * 2048 * 2
    assert pl["alg_bytes"] == 64 * (2 * fb + fb // 4 + fb // 16 + fb // 64 + fb // 256)
    assert pl["expected_ms"] == pytest.approx(pl["alg_bytes"] / pl["probe_bus_gbs"] / 1e6,
                                              rel=1e-3)
    if pl["accepted"]:
        assert min(ms) <= 1.03 * pl["expected_ms"] + 1e-9
    else:
        assert len(ms) == 4
    assert pl["peak_device_bytes"] <= est["device_bytes"]


@pytest.mark.parametrize("tries", [2, 3])
def test_placement_search_worst_case_within_estimate(gpu, tries):
    """Every try runs (bench placement_flags=1): fresh arenas, the loser
    freed at once, so the creation peak -- measured by the stage and from
    the device's free memory -- is one ring set + the random frames over
    the stage's own footprint, within aqz_stage_estimate_memory, and the
    stage keeps one ring set."""
    import torch
    kw = dict(force_levels=5, max_batch_frames=64, layer_slots=2, placement_tries=tries)
    est = gpu.estimate_memory(C2, U16, MEAN, **kw)["device_bytes"]
    st = gpu.Stage(C2, U16, MEAN, placement_flags=1, **kw)
    pl = st.placement()
    assert len(pl["candidates_ms"]) == tries and not pl["accepted"]
    assert pl["peak_device_bytes"] <= est
    held = st.memory_usage()["device_bytes"]
    assert held <= gpu.estimate_memory(C2, U16, MEAN, force_levels=5, max_batch_frames=64,
                                       layer_slots=2)["device_bytes"]
    # one ring set is held: the arena, 64 frames x 2 layers of level 0 + the rest
    lay = [st.layout(l) for l in range(st.n_levels())]
    rings = sum(x["chunk_pitch"] * x["chunks_per_layer"] * x["layer_slots"] for x in lay)
    assert rings <= held < rings * 1.1
    # the search's peak: its random frames + a second set on top of the held one
    assert pl["peak_device_bytes"] >= held + 64 * 2048 * 2048 * 2
    st.close()
    torch.cuda.synchronize()


def test_stage_destroy_returns_device_memory(gpu):
    """A stage whose rings are a VMM arena (and whose search made and freed
    a second arena) gives every byte back when destroyed, five times over
    (DevBuf::release unmaps each 2 MiB piece)."""
    import torch
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(5):
        st = gpu.Stage(C2, U16, MEAN, force_levels=5, max_batch_frames=64, layer_slots=2,
                       placement_tries=2, placement_flags=1)
        assert st.placement()["mode"] == 3
        st.close()
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    assert free0 - free1 < (64 << 20), (free0, free1)


# z 64 -> 32 -> 16 -> 16 (xy 256 -> 32), z chunk 16: slabs align to 4
ZDIMS = [(TIME, 0, 1, 1), (SPACE, 64, 16, 1), (SPACE, 256, 64, 2), (SPACE, 256, 64, 2)]
# every ring carved from one arena of 2 MiB virtual-memory pieces
ARENA = dict(ring_arena_bytes=2 << 20, ring_malloc_flags=0x100 | (5 << 9))


@pytest.mark.parametrize("slabs", [2, 4])
def test_z_slab_import_from_vmm_arenas(gpu, slabs):
    """z-slab stages whose rings live in VMM arenas (the shipped kind of
    memory of large stages, forced here on small frames): each chunk layer
    is assembled in one stage from the others' frames by
    aqz_stage_import_frames, and equals the single-stream oracle's layer.
    Stages alternate over the visible devices, so on a node the import reads
    another GPU's arena over xGMI (grant_access maps it for the reader)."""
    from aqz.dist import z_slab
    ndev = gpu.device_count()
    n = 2 * 64
    frames = synthetic_frames(U16, n, 256, 256, 91 + slabs) & 0x0fff
    frames[70:75] = 0
    exp, fw, ldims = expected_stage_layers(ZDIMS, U16, MEAN, frames)
    planes = [d[1][1] for d in ldims]
    stages, bounds = [], []
    for r in range(slabs):
        lo, hi = z_slab(64, slabs, r, 4)
        st = gpu.Stage(ZDIMS, U16, MEAN, max_batch_frames=8, layer_slots=12,
                       z_slab=(lo, hi), device=r % ndev, **ARENA)
        for vol in range(2):
            for b in range(lo, hi, 8):
                e = min(hi, b + 8)
                st.append(frames[vol * 64 + b: vol * 64 + e])
        st.synchronize()
        stages.append(st)
        bounds.append((lo, hi))
    for (l, layer), (buf, flags) in sorted(exp.items()):
        F = stages[0].layout(l)["frames_per_layer"]
        owner = layer % slabs
        shift = 64 // planes[l]
        f = layer * F
        while f < (layer + 1) * F:
            z = f % planes[l]
            r = next(i for i, (lo, hi) in enumerate(bounds) if lo // shift <= z < hi // shift)
            run = min((layer + 1) * F, f - z + bounds[r][1] // shift) - f
            if r != owner:
                stages[owner].import_frames(stages[r], l, layer, f - layer * F, run)
            f += run
        got, gflags = stages[owner].copy_layer(l, layer)
        assert_same_pixels(got, buf, U16, f"slabs {slabs} L{l} layer{layer}")
        assert np.array_equal(gflags, flags), (l, layer)
    for st in stages:
        st.close()
