"""The multi-GPU exchange step, rehearsed on CPU with gloo at world size 2 and 3.

Each rank fills its band buffer (rt_band_rows_per_rank rows) with the global row
index of every local row (exactly the rows rt_render_bands_async would render), the
buffers are gathered to rank 0 with torch.distributed.gather -- the collective bench.py
issues over RCCL -- and rank 0 reassembles them with the same index map the HIP
unpermute kernel uses.  Every frame row must come back in place exactly once.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, h, w, band, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rust_tracer_amd.dist import band_rows_per_rank_py, local_rows
        rpr = band_rows_per_rank_py(h, band, world)
        rows = local_rows(h, band, rank, world)
        local = torch.full((rpr, w), -1.0)
        for lr, v in enumerate(rows):
            if v >= 0:
                local[lr] = float(v)
        glist = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
        dist.gather(local, gather_list=glist, dst=0)
        if rank == 0:
            gathered = torch.stack(glist)
            frame = torch.empty((h, w))
            # unpermute_kernel's map: row v <- rank (v // band) % world, local row
            for v in range(h):
                b = v // band
                r = b % world
                lr = (b // world) * band + (v - b * band)
                frame[v] = gathered[r, lr]
            ok = bool(torch.equal(frame[:, 0], torch.arange(h, dtype=torch.float32)))
            q.put(ok)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,h", [(2, 1080), (3, 117)])
def test_gather_reassembles_frame(world, h):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, h, 5, 8, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get() is True


def _worker_sub(rank, world, sub, port, h, w, band, q):
    """FramePipeline's gathered band-share groups (rust_tracer_amd/dist.py): rank r's share j
    is band rank r*S + j of a world of W*S; the rank's [S, rows, W] buffer is its one gather
    contribution, and rank 0 un-permutes the gathered buffer over W*S ranks."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rust_tracer_amd.dist import band_rows_per_rank_py, local_rows
        vworld = world * sub
        rpr = band_rows_per_rank_py(h, band, vworld)
        local = torch.full((sub, rpr, w), -1.0)
        for j in range(sub):
            for lr, v in enumerate(local_rows(h, band, rank * sub + j, vworld)):
                if v >= 0:
                    local[j, lr] = float(v)
        glist = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
        dist.gather(local, gather_list=glist, dst=0)
        if rank == 0:
            gathered = torch.stack(glist).reshape(vworld, rpr, w)  # virtual-rank-major
            frame = torch.full((h, w), -2.0)
            for v in range(h):
                b = v // band
                r = b % vworld
                lr = (b // vworld) * band + (v - b * band)
                frame[v] = gathered[r, lr]
            q.put(bool(torch.equal(frame[:, 0], torch.arange(h, dtype=torch.float32))))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,sub,h", [(2, 2, 1080), (2, 4, 117), (3, 2, 90), (4, 2, 1080), (8, 4, 1080)])
def test_gather_band_share_groups(world, sub, h):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_sub, args=(r, world, sub, port, h, 5, 8, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get() is True
