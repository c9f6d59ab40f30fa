"""Multi-GPU sharding of independent oceans, and of one ocean's
cascades and column bands when there are more GPUs than (tile, cascade) units.

The per-frame path has no exchange step: every (tile, cascade) unit's
spectrum -> IFFT -> outputs -> foam chain touches only its own data.  Tiles
(independent oceans, seeded seed + global tile index) are split into
contiguous blocks over the ranks, one process per GPU, and no collective runs
on the data path.  torch.distributed (gloo) carries only the start/stop
barrier and the max-over-ranks of the elapsed time in bench.py.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple


def shard_tiles(total_tiles: int, world: int, rank: int) -> Tuple[int, int]:
    """(first global tile, tile count) of `rank`: contiguous blocks, sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total_tiles, world)
    count = base + (1 if rank < extra else 0)
    first = rank * base + min(rank, extra)
    return first, count


@dataclass(frozen=True)
class Shard:
    """One rank's share of a job of `tiles` oceans x C cascades at N^2: global tiles
    [tile0, tile0 + tiles), cascades [casc0, casc0 + cascades) of each, and the column
    band [x0, x0 + nx) of each of those slices (ocean_set_column_band) -- or, with
    parity >= 0, the columns x = 2m + parity (ocean_set_column_parity; x0 = 0, nx = N)."""
    tile0: int
    tiles: int
    casc0: int
    cascades: int
    x0: int
    nx: int
    parity: int = -1

    def columns(self, n: int):
        """The global columns this shard computes, in its texture's column order."""
        if self.parity >= 0:
            return list(range(self.parity, n, 2))
        return list(range(self.x0, self.x0 + self.nx))


def band_granularity(n: int) -> int:
    """Column-band start/width granularity of ocean_set_column_band at N = n."""
    return min(n, max(16, 8192 // n))


PARITY_SIZES = (4096,)  # N with a column-parity row pass (ocean_set_column_parity, pass A3P)


def plan_shard(total_tiles: int, n_cascades: int, n: int, world: int, rank: int, interleave: bool = True) -> Shard:
    """Split a job over `world` GPUs with no data exchange.

    world <= tiles: contiguous tile blocks, every cascade, whole slices (cfg4).
    Otherwise each tile gets s = world / tiles ranks (world a multiple of tiles):
    s <= C: the tile's cascades in contiguous blocks (cfg5 at 2 and 4 GPUs);
    s > C (s a multiple of C): each cascade over b = s / C ranks.  b = 2 at an N with the
    parity row pass (cfg5 at 8 GPUs) and `interleave`: even / odd columns (rank k of the
    cascade owns x = 2m + k; each rank transforms its rows at N/2 points instead of
    duplicating the N-point row transform).  Otherwise b column bands of N / b columns
    (every band rank runs the full row IFFT of its cascade)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    if world <= total_tiles:
        t0, nt = shard_tiles(total_tiles, world, rank)
        return Shard(t0, nt, 0, n_cascades, 0, n)
    if world % total_tiles:
        raise ValueError(f"{world} ranks over {total_tiles} tiles: world must be a multiple of the tile count")
    s = world // total_tiles
    tile, r = divmod(rank, s)
    if s <= n_cascades:
        c0, nc = shard_tiles(n_cascades, s, r)
        return Shard(tile, 1, c0, nc, 0, n)
    if s % n_cascades:
        raise ValueError(f"{s} ranks per tile over {n_cascades} cascades: must be a multiple")
    b = s // n_cascades
    c, k = divmod(r, b)
    if b == 2 and interleave and n in PARITY_SIZES:
        return Shard(tile, 1, c, 1, 0, n, parity=k)
    width = n // b
    if width < band_granularity(n) or width % band_granularity(n):
        raise ValueError(f"{b} column bands of N = {n} are narrower than the band granularity")
    return Shard(tile, 1, c, 1, k * width, width)


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
