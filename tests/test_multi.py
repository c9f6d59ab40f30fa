"""Multi-process (world_size 2, gloo, CPU) tests of the sharding used by bench.py
for BASELINE cfg4 (256 independent tiles over the GPUs of one node).  The data
path has no collective: only the barrier, max-elapsed and
tile-count reductions run over torch.distributed."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from ocean_hip.shard import Shard, band_granularity, plan_shard, reduce_timing, shard_tiles, tile_seed


@pytest.mark.parametrize("total,world", [(256, 8), (256, 2), (7, 3), (3, 4), (1, 1)])
def test_shards_cover_every_tile_once(total, world):
    seen = []
    for r in range(world):
        first, count = shard_tiles(total, world, r)
        seen.extend(range(first, first + count))
    assert seen == list(range(total))
    counts = [shard_tiles(total, world, r)[1] for r in range(world)]
    assert max(counts) - min(counts) <= 1


def test_tile_seed_is_global():
    # rank 1 of 2 over 256 tiles starts at global tile 128: seed 20251121 + 128
    first, _ = shard_tiles(256, 2, 1)
    assert tile_seed(20251121, first) == 20251121 + 128


def _cover(total_tiles, cascades, n, world, interleave=True):
    """Every (tile, cascade, column) exactly once over the ranks' shards."""
    seen = {}
    for r in range(world):
        sh = plan_shard(total_tiles, cascades, n, world, r, interleave)
        for t in range(sh.tile0, sh.tile0 + sh.tiles):
            for c in range(sh.casc0, sh.casc0 + sh.cascades):
                for x in sh.columns(n):
                    seen[(t, c, x)] = seen.get((t, c, x), 0) + 1
    return seen


@pytest.mark.parametrize("interleave", [True, False])
@pytest.mark.parametrize("tiles,cascades,n,world", [
    (256, 4, 512, 8),   # cfg4: tile blocks
    (1, 4, 4096, 1), (1, 4, 4096, 2), (1, 4, 4096, 4), (1, 4, 4096, 8),  # cfg5 at 1/2/4/8 GPUs
    (1, 4, 1024, 16), (2, 4, 1024, 8), (1, 3, 256, 3), (1, 4, 4096, 3), (1, 2, 4096, 8)])
def test_plan_covers_every_texel_once(tiles, cascades, n, world, interleave):
    seen = _cover(tiles, cascades, n, world, interleave)
    assert len(seen) == tiles * cascades * n and set(seen.values()) == {1}


def test_plan_cfg5_eight_gpus_is_even_odd_columns():
    """cfg5 on 8 GPUs: each cascade's two ranks own its even / odd columns (column parity); the
    contiguous half bands remain the plan without interleaving and past two ranks per cascade."""
    shards = [plan_shard(1, 4, 4096, 8, r) for r in range(8)]
    assert shards[0] == Shard(0, 1, 0, 1, 0, 4096, 0) and shards[1] == Shard(0, 1, 0, 1, 0, 4096, 1)
    assert shards[7] == Shard(0, 1, 3, 1, 0, 4096, 1)
    assert shards[6].columns(4096)[:3] == [0, 2, 4] and shards[7].columns(4096)[-1] == 4095
    bands = [plan_shard(1, 4, 4096, 8, r, interleave=False) for r in range(8)]
    assert bands[0] == Shard(0, 1, 0, 1, 0, 2048) and bands[1] == Shard(0, 1, 0, 1, 2048, 2048)
    assert bands[7] == Shard(0, 1, 3, 1, 2048, 2048)
    for sh in bands:
        assert sh.x0 % band_granularity(4096) == 0 and sh.nx % band_granularity(4096) == 0
    quarters = [plan_shard(1, 2, 4096, 8, r) for r in range(8)]  # 4 ranks per cascade: bands
    assert all(sh.parity == -1 and sh.nx == 1024 for sh in quarters)


@pytest.mark.parametrize("tiles,cascades,n,world", [(3, 4, 1024, 4), (1, 3, 1024, 4), (1, 1, 64, 2)])
def test_plan_rejects_uneven_splits(tiles, cascades, n, world):
    with pytest.raises(ValueError):
        plan_shard(tiles, cascades, n, world, 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, tiles = shard_tiles(256, world, rank)
    band = plan_shard(1, 1, 4096, world, rank, interleave=False)  # one 4096^2 cascade in two column bands
    par = plan_shard(1, 1, 4096, world, rank)  # ... or in its even / odd columns
    dist.barrier()
    elapsed, total = reduce_timing(0.5 + rank, tiles, world)
    q.put((rank, first, tiles, elapsed, total, band.x0, band.nx, par.parity))
    dist.destroy_process_group()


def test_gloo_world2_barrier_and_reductions():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [o[1:3] for o in out] == [(0, 128), (128, 128)]
    for o in out:
        assert o[3] == 1.5 and o[4] == 256  # max elapsed, summed tiles on every rank
    assert [o[5:7] for o in out] == [(0, 2048), (2048, 2048)]
    assert [o[7] for o in out] == [0, 1]
