"""Patch sharding, the final objCrop gather and stitching.

Patches are independent FPM problems (the per-LED crop offsets depend only on
the LED position, fpmMain.cpp:146-168), so a field of P patches is split into
contiguous blocks, one per rank, with no collective inside an iteration.  The
only exchange is one gather of every rank's high-resolution tiles to rank 0
after the last iteration, followed by placing tile i at its (row, column) of
the patch grid: tiles do not overlap, so stitching is pure placement.  The
reference processes a single patch, so stitching is new here.

torch.distributed carries the gather (backend "nccl" = RCCL over xGMI on the
GPU box, "gloo" in the CPU tests); nothing here touches the solver itself.
"""
from __future__ import annotations

import numpy as np


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Half-open patch range [lo, hi) owned by `rank`: contiguous blocks of
    ceil(total/world), the last rank taking the remainder (possibly empty)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    per = -(-total // world)
    lo = min(total, rank * per)
    return lo, min(total, lo + per)


def gather_tiles(tiles, dist, dst: int = 0):
    """Gather every rank's [n_local, L, L, 2] float32 tiles onto `dst`.

    Ranks may own different patch counts (the last shard can be short), so the
    local tensor is padded to the largest shard; rank `dst` returns the
    concatenation in rank order with the padding dropped, other ranks None."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    n = torch.tensor([tiles.shape[0]], dtype=torch.int64, device=tiles.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    nmax = max(counts)
    if tiles.shape[0] < nmax:
        pad = torch.zeros((nmax - tiles.shape[0],) + tuple(tiles.shape[1:]), dtype=tiles.dtype, device=tiles.device)
        tiles = torch.cat([tiles, pad])
    bufs = [torch.empty_like(tiles) for _ in range(world)] if rank == dst else None
    dist.gather(tiles.contiguous(), bufs, dst=dst)
    if rank != dst:
        return None
    return torch.cat([b[:c] for b, c in zip(bufs, counts)])


def field_grid(total: int) -> tuple[int, int]:
    """(gy, gx) of the most nearly square grid with gy * gx == total, gy <= gx
    (1024 patches -> 32 x 32)."""
    gy = int(total ** 0.5)
    while gy > 1 and total % gy:
        gy -= 1
    return max(gy, 1), total // max(gy, 1)


def stitch(tiles, grid: tuple[int, int]):
    """Place tiles [P, L, L(, 2)] (row-major patch order) on a grid (gy, gx):
    tile i lands at rows (i // gx)*L and columns (i % gx)*L.  numpy arrays
    and torch tensors (e.g. the gathered tiles still on rank 0's GPU) alike."""
    gy, gx = grid
    P, L = tiles.shape[0], tiles.shape[1]
    if P != gy * gx:
        raise ValueError(f"{P} tiles for a {gy}x{gx} grid")
    rest = tuple(tiles.shape[3:])
    out = tiles.reshape((gy, gx, L, L) + rest).swapaxes(1, 2).reshape((gy * L, gx * L) + rest)
    return np.ascontiguousarray(out) if isinstance(out, np.ndarray) else out.contiguous()
