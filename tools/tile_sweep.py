#!/usr/bin/env python3
"""Wide vs narrow (4-column) tiles of the fused path on small jobs: pass A + pass B
kernel time per frame for each (N, cascades, planes); OCEAN_TILE_W picks the width
at ocean_create (docs/MEASUREMENTS.md section 3, narrow tiles)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ocean-simulation_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import torch  # noqa: F401,E402
import ocean_hip as oh  # noqa: E402
from oracle import SCENE_CASCADES, scene_params  # noqa: E402

WIDE = {128: "64", 256: "32", 512: "16", 1024: "8"}  # inter_w(N), fft_core.h


def run(n, C, flags, width):
    os.environ["OCEAN_TILE_W"] = width
    cas = (SCENE_CASCADES * 2)[:C]
    c = oh.OceanContext(n, C, 1, flags)
    c.set_params(scene_params(), cas)
    c.generate_noise(1)
    c.init_spectrum()
    for f in range(20):
        c.step(f / 60)
    c.synchronize()
    c.set_kernel_timing(True)
    c.kernel_stats(0), c.kernel_stats(1)
    K = 200
    for f in range(K):
        c.step(f / 60)
    a_ms, _ = c.kernel_stats(0)
    b_ms, _ = c.kernel_stats(1)
    c.close()
    return 1e3 * a_ms / K, 1e3 * b_ms / K


cases = [(512, 1, oh.F_DISPLACEMENT_ONLY), (512, 1, 0), (512, 2, 0), (512, 3, 0), (512, 4, 0),
         (1024, 1, oh.F_DISPLACEMENT_ONLY), (1024, 1, 0), (256, 1, 0), (256, 4, 0), (128, 4, 0)]
for n, C, flags in cases:
    wa, wb = run(n, C, flags, WIDE[n])
    na, nb = run(n, C, flags, "4")
    print(f"N={n} C={C} P={2 if flags else 4}: wide A {wa:.2f} B {wb:.2f} = {wa + wb:.2f} us; "
          f"narrow A {na:.2f} B {nb:.2f} = {na + nb:.2f} us", flush=True)
