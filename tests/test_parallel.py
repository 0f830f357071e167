"""Patch sharding / gather / stitch (fpm_amd.parallel) on CPU: world size 2
over gloo with 127.0.0.1 rendezvous, the N > 1 path of bench.py without a GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fpm_amd import parallel


def test_shard_range_covers_everything():
    for total in (0, 1, 7, 256, 1023, 1024):
        for world in (1, 2, 3, 4, 8):
            seen = []
            for r in range(world):
                lo, hi = parallel.shard_range(total, world, r)
                assert 0 <= lo <= hi <= total
                seen.extend(range(lo, hi))
            assert seen == list(range(total))
    with pytest.raises(ValueError):
        parallel.shard_range(4, 2, 2)


def test_stitch_places_tiles():
    L, gy, gx = 4, 2, 3
    tiles = np.arange(gy * gx * L * L * 2, dtype=np.float32).reshape(gy * gx, L, L, 2)
    f = parallel.stitch(tiles, (gy, gx))
    assert f.shape == (gy * L, gx * L, 2)
    for i in range(gy * gx):
        r, c = divmod(i, gx)
        np.testing.assert_array_equal(f[r * L:(r + 1) * L, c * L:(c + 1) * L], tiles[i])
    with pytest.raises(ValueError):
        parallel.stitch(tiles, (4, 4))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, L, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = parallel.shard_range(total, world, rank)
    # each rank "reconstructs" its own patches: tile value encodes patch index
    idx = torch.arange(lo, hi, dtype=torch.float32)
    tiles = idx[:, None, None, None].expand(hi - lo, L, L, 2).contiguous()
    out = parallel.gather_tiles(tiles, dist)
    if rank == 0:
        q.put(out.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [6, 5])
def test_gather_world2_gloo(total):
    world, L = 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, L, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert got.shape == (total, L, L, 2)
    np.testing.assert_array_equal(got[:, 0, 0, 0], np.arange(total, dtype=np.float32))
    field = parallel.stitch(got[:6] if total == 6 else np.concatenate([got, got[:1]]), (2, 3))
    assert field.shape == (2 * L, 3 * L, 2)
