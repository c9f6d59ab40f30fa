"""Multi-GPU sharding of independent oceans.

The per-frame path has no exchange step: every (tile, cascade) unit's
spectrum -> IFFT -> outputs -> foam chain touches only its own data.  Tiles
(independent oceans, seeded seed + global tile index) are split into
contiguous blocks over the ranks, one process per GPU, and no collective runs
on the data path.  torch.distributed (gloo) carries only the start/stop
barrier and the max-over-ranks of the elapsed time in bench.py.
"""
from __future__ import annotations

from typing import Tuple


def shard_tiles(total_tiles: int, world: int, rank: int) -> Tuple[int, int]:
    """(first global tile, tile count) of `rank`: contiguous blocks, sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total_tiles, world)
    count = base + (1 if rank < extra else 0)
    first = rank * base + min(rank, extra)
    return first, count


def tile_seed(seed: int, global_tile: int) -> int:
    """Noise seed of a global tile (ocean_generate_noise uses seed + local tile)."""
    return seed + global_tile


def reduce_timing(elapsed: float, tiles: int, world: int):
    """Max elapsed and total tiles over ranks (gloo, CPU tensors); identity when world == 1."""
    if world == 1:
        return elapsed, tiles
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    n = torch.tensor([tiles], dtype=torch.int64)
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    return float(t[0]), int(n[0])
