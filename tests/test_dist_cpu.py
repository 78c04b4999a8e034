"""CPU suite, part 3: the N>1 path, world_size 2 over gloo.

The stage shards without a data-path collective (aqz/dist.py): 2-D configs
run one independent stream per GPU; the 3-D config splits z into aligned
slabs.  Here two gloo ranks (a) run the bench's timed-region protocol
(barrier + max over ranks) and (b) each downsample one z slab of a volume
with the oracle; the gathered slabs must equal the single-process pyramid.
"""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aqz.dist import timed_region, torch_reduce_max, z_levels, z_slab
import oracle_bindings as ob


def test_z_slab_partition():
    for n, world, align in [(256, 4, 4), (256, 8, 4), (100, 3, 4), (64, 2, 8), (7, 2, 2)]:
        spans = [z_slab(n, world, r, align) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        for (a, b), (c, d) in zip(spans, spans[1:]):
            assert b == c
        for lo, hi in spans:
            assert lo % align == 0 and lo <= hi
    assert z_levels([256, 128, 64, 64]) == 2
    assert z_slab(256, 4, 1, 4) == (64, 128)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # (a) timed region: rank 1 is slower; both must report its time
        def step(s):
            time.sleep(0.002 * (1 + 4 * rank))
        el = timed_region(step, steps=5, warmup=1, sync=lambda: None,
                          barrier=dist.barrier,
                          reduce_max=torch_reduce_max(dist, torch.device("cpu")))
        # (b) z-slab sharded pyramid of a 3-D volume
        Z, H, W = 32, 24, 20
        dims = [(ob.TIME, 0, 1, 1), (ob.SPACE, Z, 4, 1), (ob.SPACE, H, 6, 1),
                (ob.SPACE, W, 5, 1)]
        vol = ob.synthetic_frames(ob.U16, Z, H, W, 321)
        ds = ob.OracleDownsampler(dims, ob.U16, ob.MEAN)
        planes = [ds.level_dims(l)[1][1] for l in range(ds.n_levels())]
        lo, hi = z_slab(Z, world, rank, 1 << z_levels(planes))
        outs = {l: [] for l in range(1, ds.n_levels())}
        for z in range(lo, hi):
            ds.add_frame(vol[z])
            for l in outs:
                img = ds.take_frame(l)
                if img is not None:
                    outs[l].append(img)
        gathered = {}
        for l, imgs in outs.items():
            t = torch.from_numpy(np.stack(imgs).astype(np.int32)) if imgs else \
                torch.zeros((0, 1, 1), dtype=torch.int32)
            n = torch.tensor([t.shape[0]])
            ns = [torch.zeros_like(n) for _ in range(world)]
            dist.all_gather(ns, n)
            buf = [torch.zeros((int(k.item()),) + tuple(t.shape[1:]), dtype=torch.int32)
                   for k in ns]
            dist.all_gather(buf, t)
            gathered[l] = torch.cat(buf).numpy().astype(np.uint16)
        if rank == 0:
            full = ob.OracleDownsampler(dims, ob.U16, ob.MEAN)
            ref = {l: [] for l in outs}
            for z in range(Z):
                full.add_frame(vol[z])
                for l in ref:
                    img = full.take_frame(l)
                    if img is not None:
                        ref[l].append(img)
            ok = all(np.array_equal(gathered[l], np.stack(ref[l])) for l in ref)
            q.put((el, ok, {l: len(ref[l]) for l in ref}))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_rank_gloo_timing_and_z_slab_sharding():
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, q), nprocs=2, join=True,
                       start_method="spawn")
    el, ok, counts = q.get()
    assert el >= 5 * 0.010 * 0.9, el  # the slow rank's time is reported
    assert ok, "z-slab sharded pyramid differs from the single-process one"
    assert counts[1] == 16 and counts[2] == 8
