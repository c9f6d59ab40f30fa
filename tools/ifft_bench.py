#!/usr/bin/env python3
"""Operator-level IFFT timing: ocean_ifft2d over the 4 planes of a 4 x 1024^2 context,
per-launch-kind averages from the library's HIP-event timing (kind 0 = row launches,
kind 1 = column launches).  Used for A/B runs of the unfused kernels:
    python tools/ifft_bench.py [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ocean-simulation_amd"))
import torch  # noqa: F401,E402  (one HIP runtime: torch's)
import ocean_hip as oh  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
n, C = 1024, 4
ctx = oh.OceanContext(n, C, 1, 0)
for _ in range(5):
    ctx.ifft2d(0b1111)
ctx.synchronize()
ctx.set_kernel_timing(True)
ctx.kernel_stats(0), ctx.kernel_stats(1)
for _ in range(reps):
    ctx.ifft2d(0b1111)
ctx.synchronize()
r_ms, r_n = ctx.kernel_stats(0)
c_ms, c_n = ctx.kernel_stats(1)
plane_bytes = n * n * C * 8
rows_us = 1e3 * r_ms / reps
cols_us = 1e3 * c_ms / reps
out = {"rows_us": round(rows_us, 2), "cols_us": round(cols_us, 2), "row_launches": r_n // reps,
       "col_launches": c_n // reps,
       "rows_GBs": round(2 * 4 * plane_bytes / (rows_us * 1e-6) / 1e9, 1),
       "cols_GBs": round(2 * 4 * plane_bytes / (cols_us * 1e-6) / 1e9, 1),
       "stage_GBs": round(4 * 4 * plane_bytes / ((rows_us + cols_us) * 1e-6) / 1e9, 1)}
print(json.dumps(out))
