#!/usr/bin/env python3
"""Three-plane vs four-plane fused frame (OCEAN_Q=1 / 0, read at ocean_create) on a set of
(N, cascades, tiles) shapes: pass A + pass B kernel time per frame by the library's dispatch
events, and wall time per frame (three-plane frame).
    python tools/q_sweep.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ocean-simulation_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import torch  # noqa: F401,E402
import ocean_hip as oh  # noqa: E402
from oracle import SCENE_CASCADES, scene_params  # noqa: E402


def run(n, C, T, q):
    os.environ["OCEAN_Q"] = str(q)
    cas = (SCENE_CASCADES * 2)[:C]
    c = oh.OceanContext(n, C, T, 0)
    c.set_params(scene_params(), cas)
    c.generate_noise_device(1)
    c.init_spectrum()
    for f in range(20):
        c.step(f / 60)
    c.synchronize()
    K = 300
    t0 = time.perf_counter()
    for f in range(K):
        c.step((20 + f) / 60)
    c.synchronize()
    wall = (time.perf_counter() - t0) / K * 1e6
    c.set_kernel_timing(True)
    c.kernel_stats(0), c.kernel_stats(1)
    for f in range(K):
        c.step((20 + K + f) / 60)
    a_ms, _ = c.kernel_stats(0)
    b_ms, _ = c.kernel_stats(1)
    c.close()
    return {"a_us": round(a_ms * 1e3 / K, 2), "b_us": round(b_ms * 1e3 / K, 2), "wall_us": round(wall, 2)}


for n, C, T in [tuple(map(int, s.split("x"))) for s in (sys.argv[1:] or ["512x1x1", "512x3x1", "512x4x1", "512x4x8", "1024x1x1", "1024x2x1", "1024x4x1", "1024x4x4", "2048x4x1"])]:
    r = {q: run(n, C, T, q) for q in (1, 0)}
    print(json.dumps({"n": n, "cascades": C, "tiles": T, "q": r[1], "four_plane": r[0]}), flush=True)
