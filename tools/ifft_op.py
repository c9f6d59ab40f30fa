#!/usr/bin/env python3
"""Operator-level IFFT (ocean_ifft2d, IFFT.InverseFastFourierTransform) timing at any shape:
per-launch-kind averages from the library's HIP-event timing (kind 0 = row launches, kind 1 =
column launches) and the wall time of the whole 4-plane operator.
    python tools/ifft_op.py N C T [reps] [mask]
One JSON line: algorithmic bytes 32 B per texel per plane (read + write, two passes)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ocean-simulation_amd"))
import torch  # noqa: F401,E402  (one HIP runtime: torch's)
import ocean_hip as oh  # noqa: E402

n, C, T = (int(a) for a in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 50
mask = int(sys.argv[5]) if len(sys.argv) > 5 else 0b1111
planes = bin(mask).count("1")
ctx = oh.OceanContext(n, C, T, oh.F_UNFUSED)
# the frame's own data in the planes (zero-filled planes run at a higher clock, MI355X_MICROARCH.md)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
ctx.set_params(bench.SCENE_PARAMS, (bench.SCENE_CASCADES * 2)[:C])
ctx.generate_noise_device(20251121)
ctx.init_spectrum()
for k in range(5):
    ctx.evolve(0.1 * k)
    ctx.ifft2d(mask)
ctx.synchronize()
# every call on freshly evolved planes (the unnormalised inverse transform overflows to inf / NaN
# within a dozen calls); wall = (evolve + operator) - (evolve alone)
t0 = time.perf_counter()
for k in range(reps):
    ctx.evolve(0.5 + k / 60.0)
    ctx.ifft2d(mask)
ctx.synchronize()
t1 = time.perf_counter()
for k in range(reps):
    ctx.evolve(0.5 + k / 60.0)
ctx.synchronize()
t2 = time.perf_counter()
wall_us = 1e6 * ((t1 - t0) - (t2 - t1)) / reps
ctx.set_kernel_timing(True)
ctx.kernel_stats(0), ctx.kernel_stats(1), ctx.kernel_stats(2)
for k in range(reps):
    ctx.evolve(0.5 + k / 60.0)
    ctx.ifft2d(mask)
ctx.synchronize()
r_ms, r_n = ctx.kernel_stats(0)
c_ms, c_n = ctx.kernel_stats(1)
ctx.set_kernel_timing(False)
pass_bytes = 16 * n * n * C * T * planes
rows_us = 1e3 * r_ms / reps
cols_us = 1e3 * c_ms / reps
print(json.dumps({
    "n": n, "C": C, "T": T, "mask": mask, "plane_MiB": n * n * C * T * 8 * planes / 2**20,
    "rows_us": round(rows_us, 2), "cols_us": round(cols_us, 2), "wall_us": round(wall_us, 2),
    "row_launches": r_n // reps, "col_launches": c_n // reps,
    "rows_frac": round(pass_bytes / (rows_us * 1e-6) / 8e12, 4),
    "cols_frac": round(pass_bytes / (cols_us * 1e-6) / 8e12, 4),
    "kernel_frac": round(2 * pass_bytes / ((rows_us + cols_us) * 1e-6) / 8e12, 4),
    "wall_frac": round(2 * pass_bytes / (wall_us * 1e-6) / 8e12, 4)}), flush=True)
ctx.close()
