#!/usr/bin/env python3
"""Concurrency probe: K independent cfg3 oceans, each on its own HIP stream, stepped
round-robin.  Frames/s over all oceans vs one ocean shows how much of pass A (latency-
bound) the hardware overlaps with another ocean's pass B (bandwidth-bound)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ocean-simulation_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import torch  # noqa: F401,E402
import ocean_hip as oh  # noqa: E402
from oracle import SCENE_CASCADES, scene_params  # noqa: E402

steps = 200
for k in (1, 2, 3):
    ctxs = []
    for i in range(k):
        c = oh.OceanContext(1024, 4, 1, 0)
        c.set_params(scene_params(), SCENE_CASCADES)
        c.generate_noise(100 + i)
        c.init_spectrum()
        ctxs.append(c)
    for f in range(20):
        for c in ctxs:
            c.step(f / 60)
    for c in ctxs:
        c.synchronize()
    t0 = time.perf_counter()
    for f in range(steps):
        for c in ctxs:
            c.step(f / 60)
    for c in ctxs:
        c.synchronize()
    dt = time.perf_counter() - t0
    print(f"{k} oceans: {k * steps / dt:.0f} ocean-frames/s, {1e6 * dt / steps:.1f} us per round", flush=True)
    for c in ctxs:
        c.close()
