"""Multi-GPU plumbing for the stage: one process per GPU, no data-path
collective.

The pyramid shards by independent units:
  * 2-D configs: every GPU runs its own camera/frame stream (weak scaling);
  * the 3-D light-sheet config: the volume's z planes are split into slabs,
    one per GPU, each slab a multiple of 2**(z-halving levels) planes so a
    z pair (and every deeper z group) never straddles two GPUs.  A slab's
    stage is created with first_frame = its first plane so every level's
    tiles land at their global chunk offsets; the host assembles chunk layers
    from the per-GPU pieces (no collective, no halo).
The only cross-rank operations are the bench's barrier and the max of the
timed region.
"""
from __future__ import annotations

import time
from typing import Callable, Optional, Tuple


def z_levels(planes_per_level) -> int:
    """Number of levels at which the z extent halves."""
    n = 0
    for a, b in zip(planes_per_level, planes_per_level[1:]):
        if b < a:
            n += 1
    return n


def z_slab(n_planes: int, world: int, rank: int, align: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) planes of `rank`, every boundary a multiple of
    `align` (= 2**z_levels); the last rank takes the remainder."""
    if align <= 0 or world <= 0 or not 0 <= rank < world:
        raise ValueError("bad slab arguments")
    groups = -(-n_planes // align)
    per = groups // world
    extra = groups % world
    g_lo = rank * per + min(rank, extra)
    g_hi = g_lo + per + (1 if rank < extra else 0)
    return min(n_planes, g_lo * align), min(n_planes, g_hi * align)


def timed_region(step: Callable[[int], None], steps: int, warmup: int,
                 sync: Callable[[], None], barrier: Optional[Callable[[], None]],
                 reduce_max: Optional[Callable[[float], float]]) -> float:
    """W untimed steps, then EXACTLY `steps` steps bracketed by barrier +
    device sync on both sides; returns the max over ranks of the elapsed
    seconds (the bench contract)."""
    for s in range(warmup):
        step(s)
    sync()
    if barrier:
        barrier()
    sync()
    t0 = time.perf_counter()
    for s in range(steps):
        step(warmup + s)
    sync()
    t1 = time.perf_counter()
    if barrier:
        barrier()
    elapsed = t1 - t0
    return reduce_max(elapsed) if reduce_max else elapsed


def torch_reduce_max(dist, device):
    import torch

    def f(x: float) -> float:
        t = torch.tensor([x], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    return f
