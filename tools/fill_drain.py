#!/usr/bin/env python3
"""Per-launch fill/drain estimate: kernel times at C = 1, 2, 4 cascades of 1024^2
(the same per-workgroup work repeated 1, 2, 4 times); t(C) ~ fixed + C * per_unit.
    python tools/fill_drain.py [C or CxT ...]   (default 1 2 4; T tiles of C cascades)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ocean-simulation_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import torch  # noqa: F401,E402
import ocean_hip as oh  # noqa: E402
from oracle import SCENE_CASCADES, scene_params  # noqa: E402

for arg in sys.argv[1:] or ["1", "2", "4"]:
    C, T = (list(map(int, arg.split("x"))) + [1])[:2]
    cas = (SCENE_CASCADES * 2)[:C]
    c = oh.OceanContext(1024, C, T, 0)
    c.set_params(scene_params(), cas)
    c.generate_noise_device(1)
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
    print(f"C={C} T={T} units={C * T}: pass A {1e3 * a_ms / K:.2f} us, pass B {1e3 * b_ms / K:.2f} us", flush=True)
    c.close()
