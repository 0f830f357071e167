"""Multi-rank path on one GPU: two gloo ranks, each solving
its own contiguous shard of a 2 x 3 patch field with the HIP solver on the
same MI355X, one gather of the objCrop tiles to rank 0, stitch -- the
stitched field must equal a single-rank reconstruction of all six patches
bit for bit (patches are independent; shards change nothing inside a patch).

Inputs are seeded per GLOBAL patch index (tools/synth.make_stack seeds patch
b with seed + b), so a shard's data does not depend on the shard layout.
The fused (Np 256), the small-patch fused (Np 64) and the general (Np 64,
forced) paths are covered.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GRID = (2, 3)
TOTAL = GRID[0] * GRID[1]
CASES = {
    "fused": dict(Np=256, L=512, r=20, n_side=3, step=24, d1=10, d2=3, iters=1),
    "general": dict(Np=64, L=192, r=10, n_side=5, step=6, d1=5, d2=10, iters=2, general=True),
    "small": dict(Np=64, L=192, r=10, n_side=5, step=6, d1=5, d2=10, iters=2),  # small-patch fused kernel
}
SEED = 7100


def _problem(c, n_patch):
    import fpm_amd
    from tools.synth import grid_geometry
    x0, y0, order = grid_geometry(c["Np"], c["L"], c["n_side"], c["step"])
    path = fpm_amd.PATH_GENERAL if c.get("general") else fpm_amd.PATH_AUTO
    return fpm_amd.Problem(c["Np"], c["L"], order, x0, y0, c["r"], c["d1"], c["d2"], n_patch=n_patch,
                           path=path), x0, y0


def _solve(c, lo, hi):
    import fpm_amd
    from tools.synth import make_stack
    prob, x0, y0 = _problem(c, hi - lo)
    stack = make_stack(c["Np"], c["L"], c["r"], x0, y0, n_patch=hi - lo, seed=SEED + lo)
    with fpm_amd.Solver(prob) as s:
        s.upload(stack)
        s.init()
        s.run(c["iters"])
        return s.download(objF=False, pupil=False, support=False)["objCrop"], s.info().path


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, name, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "tests"), os.path.join(root, "fpm-opencv_amd", "python")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from fpm_amd import parallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = parallel.shard_range(TOTAL, world, rank)
        tiles, path = _solve(CASES[name], lo, hi)
        t = torch.from_numpy(np.ascontiguousarray(tiles).view(np.float32).reshape(hi - lo, *tiles.shape[1:], 2))
        got = parallel.gather_tiles(t, dist, dst=0)
        if rank == 0:
            q.put((path, parallel.stitch(got.numpy(), GRID)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["fused", "general", "small"])
def test_two_ranks_stitched_field_equals_single_rank(name):
    import torch.multiprocessing as mp
    import fpm_amd
    from fpm_amd import parallel
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    path, field = q.get()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    want_path = fpm_amd.PATH_GENERAL if name == "general" else fpm_amd.PATH_FUSED
    assert path == want_path
    tiles, path1 = _solve(CASES[name], 0, TOTAL)
    assert path1 == want_path
    ref = parallel.stitch(np.ascontiguousarray(tiles).view(np.float32).reshape(TOTAL, *tiles.shape[1:], 2), GRID)
    assert field.shape == ref.shape == (GRID[0] * CASES[name]["L"], GRID[1] * CASES[name]["L"], 2)
    np.testing.assert_array_equal(field, ref)
