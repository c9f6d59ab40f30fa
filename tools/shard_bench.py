#!/usr/bin/env python3
"""Per-shard frame times of a split job, measured one shard at a time on ONE GPU.

    python tools/shard_bench.py [--config cfg5] [--worlds 1,2,4,8] [--steps 100]

For every world size W and every rank r of ocean_hip.shard.plan_shard's W-way split
(cfg5: cascade blocks, then column bands), builds that rank's context alone on
cuda:0 and times K frames of it (ocean_step, barrier-free, synchronize on both
sides).  Ranks of a split share nothing (no data exchange), so on a node with W
GPUs the job's frame time is the slowest shard's: the printed
projected_frames_per_s = 1 / max over ranks.  This is a projection from
single-GPU measurements, not a multi-GPU measurement (bench.py --gpus W under
torchrun is that); it tells how well the split balances and what the duplicated
row pass of a column band costs.  One JSON line per world size.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ocean-simulation_amd"))

import torch  # noqa: E402,F401  (one HIP runtime per process: torch first)

import bench  # noqa: E402
import ocean_hip as oh  # noqa: E402
from ocean_hip.shard import plan_shard, tile_seed  # noqa: E402


def time_shard(cfg, sh, steps, warmup):
    n = cfg["n"]
    ctx = oh.OceanContext(n, sh.cascades, sh.tiles, 0)
    ctx.set_params(bench.SCENE_PARAMS, bench.SCENE_CASCADES[sh.casc0:sh.casc0 + sh.cascades])
    ctx.generate_noise(tile_seed(20251121, sh.tile0))
    if sh.parity >= 0:
        ctx.set_column_parity(sh.parity)
    elif sh.nx != n:
        ctx.set_column_band(sh.x0, sh.nx)
    ctx.init_spectrum()
    for f in range(warmup):
        ctx.step(f / 60.0)
    ctx.synchronize()
    t0 = time.perf_counter()
    for f in range(steps):
        ctx.step((warmup + f) / 60.0)
    ctx.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / steps
    ctx.set_kernel_timing(True)
    ctx.kernel_stats(0), ctx.kernel_stats(1)
    for f in range(steps):
        ctx.step((warmup + steps + f) / 60.0)
    a_ms, _ = ctx.kernel_stats(0)
    b_ms, _ = ctx.kernel_stats(1)
    a, b = ctx.step_bytes()
    ctx.close()
    return {"cascades": [sh.casc0, sh.casc0 + sh.cascades],
            "columns": f"x = 2m + {sh.parity}" if sh.parity >= 0 else [sh.x0, sh.x0 + sh.nx],
            "tiles": sh.tiles, "ms_per_frame": round(ms, 4),
            "pass_a_ms": round(a_ms / steps, 4), "pass_b_ms": round(b_ms / steps, 4),
            "bytes_per_frame": a + b}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg5", choices=["cfg4", "cfg5"])
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-interleave", action="store_true", help="contiguous column bands instead of even / odd")
    ap.add_argument("--all-ranks", action="store_true",
                    help="time every rank (default: one rank per distinct shard shape)")
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    for w in [int(x) for x in args.worlds.split(",")]:
        shards = [plan_shard(cfg["tiles"], cfg["cascades"], cfg["n"], w, r, not args.no_interleave) for r in range(w)]
        seen, ranks = set(), []
        for r, sh in enumerate(shards):
            # cascade sets differ in spectrum content but not in work: one per (count, band width) shape
            shape = (sh.tiles, sh.cascades, sh.nx, sh.parity)
            if args.all_ranks or shape not in seen:
                seen.add(shape)
                ranks.append(r)
        res = {r: time_shard(cfg, shards[r], args.steps, args.warmup) for r in ranks}
        worst = max(v["ms_per_frame"] for v in res.values())
        print(json.dumps({"config": args.config, "world": w, "timed_ranks": ranks,
                          "shards": {str(r): v for r, v in res.items()},
                          "projected_frames_per_s": round(cfg["tiles"] * 1e3 / worst, 2),
                          "note": "per-shard times measured alone on one MI355X; projection = 1 / slowest shard"}),
              flush=True)


if __name__ == "__main__":
    main()
