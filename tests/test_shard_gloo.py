"""Multi-GPU path on the CPU: row sharding + the gather-to-rank-0 exchange,
run with world_size 2 and 3 over gloo.  The per-rank rows come from the Tier-B
oracle (a stand-in for the GPU kernel, which is bit-identical to it — see
test_gpu_parity.py::test_row_shards_are_bit_identical_to_full_image)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rtw_amd.shard import assemble, gather_image, max_rows, shard_rows

W, H, SPP = 40, 23, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
        import rtw_oracle as O
        sc, _ = O.cover_scene(42)
        cam = O.cover_camera(16 / 9)
        rb, rs, rc = shard_rows(H, rank, world)
        rows, _ = O.render_tier_b(sc, cam, W, H, SPP, row_begin=rb, row_stride=rs, row_count=rc, threads=1)
        img = gather_image(torch.from_numpy(rows), H, rank, world)
        if rank == 0:
            q.put(img.numpy().copy())
        else:
            assert img is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_assembles_the_full_image(oracle, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    img = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sc, _ = oracle.cover_scene(42)
    full, _ = oracle.render_tier_b(sc, oracle.cover_camera(16 / 9), W, H, SPP)
    assert (img == full).all()


@pytest.mark.parametrize("height", [675, 2160, 23, 8, 1])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shard_rows_partition(height, world):
    seen = []
    for r in range(world):
        rb, rs, rc = shard_rows(height, r, world)
        rows = [rb + q * rs for q in range(rc)]
        assert all(0 <= y < height for y in rows)
        assert rc <= max_rows(height, world)
        seen += rows
    assert sorted(seen) == list(range(height))


def test_weak_scaling_balance():
    """bench.py's weak-scaling job: per-rank samples within 1% of the N=1 job."""
    base = 675 * 1200 * 500
    for world in (1, 2, 4, 8):
        per = [shard_rows(675, r, world)[2] * 1200 * 500 * world for r in range(world)]
        assert max(per) / base < 1.01


def test_assemble_single_rank():
    t = torch.arange(5 * 2 * 3, dtype=torch.uint8).reshape(5, 2, 3)
    assert torch.equal(assemble([t], 5, 1), t)
