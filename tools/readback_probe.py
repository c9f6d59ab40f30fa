#!/usr/bin/env python3
"""Where the reference Update loop's time goes at cfg3 (bench.update_loop): the
frame with mips alone, the 16 MiB snapshot readback alone (ocean_read_async into a pinned slot, waited),
the host copy-out of a completed slice alone (GetData().ToArray()), and the loop.  One JSON line.
    python tools/readback_probe.py [frames]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ocean-simulation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime: torch's)
import ocean_hip as oh  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 200
wb = oh.scene_water_body(n=1024, n_cascades=4, seed=20251121).Awake()
ctx = wb.ctx
# the probe's own pinned slots (borrowing the facade's ring capped the deepest ring at its 5 slots
# and could reuse the slot the facade's landed slice sits in)
SLOT_BYTES = 1024 * 1024 * 16
slots = [oh.PinnedBuffer(SLOT_BYTES) for _ in range(8)]
slot = slots[0]
for f in range(20):
    ctx.step(f / 60.0)
ctx.synchronize()


def timed(fn, k=frames):
    t0 = time.perf_counter()
    for f in range(k):
        fn(f)
    ctx.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


out = {"workload": "cfg3 WaterBody (mips on), ms per frame", "frames": frames}
out["step_with_mips_ms"] = timed(lambda f: ctx.step(f / 60.0))


def readback_only(f):
    rb = ctx.read_async(oh.TEX_DISP, 0, 0, slot)
    rb.wait()
    rb.release()


out["readback_16MiB_waited_ms"] = timed(readback_only)
rb = ctx.read_async(oh.TEX_DISP, 0, 0, slot)
rb.wait()
t0 = time.perf_counter()
for f in range(frames):
    _ = rb.data
out["host_copy_out_16MiB_ms"] = (time.perf_counter() - t0) / frames * 1e3
rb.release()
out["readback_GBs"] = round(16 * 2**20 / (out["readback_16MiB_waited_ms"] * 1e-3) / 1e9, 2)
out["host_copy_GBs"] = round(16 * 2**20 / (out["host_copy_out_16MiB_ms"] * 1e-3) / 1e9, 2)
out["update_loop_ms"] = timed(lambda f: wb.Update(f / 60.0))
wb.WaitForReadback()
# the readback ring alone (no frames): 8 requests in flight, the oldest waited when the ring is full
ring, idle = [], list(slots)


def ring_only(f):
    if not idle:
        r = ring.pop(0)
        r.wait()
        idle.append(r.slot)
        r.release()
    ring.append(ctx.read_async(oh.TEX_DISP, 0, 0, idle.pop()))


out["readback_ring_only_ms"] = timed(ring_only)
for r in ring:
    r.wait()
    r.release()
# the Update loop's shape at several ring depths (requests in flight), with and without the frames


def ring_loop(depth, with_step, k=frames):
    assert depth <= len(slots)
    idle_slots, q = list(slots[:depth]), []

    def finish(r):
        r.wait()
        idle_slots.append(r.slot)
        r.release()
    t0 = time.perf_counter()
    for f in range(k):
        if with_step:
            ctx.step(f / 60.0)
        while q and q[0].done():
            finish(q.pop(0))
        if not idle_slots:
            finish(q.pop(0))
        q.append(ctx.read_async(oh.TEX_DISP, 0, 0, idle_slots.pop()))
    while q:
        finish(q.pop(0))
    return (time.perf_counter() - t0) / k * 1e3


for d in (1, 2, 4, 8):
    out[f"ring{d}_readback_only_ms"] = ring_loop(d, False)
    out[f"ring{d}_with_frames_ms"] = ring_loop(d, True)
# frame + readback waited every frame (no overlap)
out["step_then_readback_waited_ms"] = timed(lambda f: (ctx.step(f / 60.0), readback_only(f)))
# host time of one Update call (the ring full: includes waiting for the oldest request)
t0 = time.perf_counter()
for f in range(frames):
    ctx.step(f / 60.0)
t_issue = (time.perf_counter() - t0) / frames * 1e3
ctx.synchronize()
out["host_issue_step_ms"] = t_issue
wb.OnDisable()
for b in slots:
    b.release()
print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}))
