"""Per-channel error report of the fused frame against the oracle for N = 16..1024 and
1 / 4 cascades (GPU).  Used to localise the gfx950 buffer_store corruption that made the
kernels use global stores (findings): the corrupted channels stand out."""
import sys, os
sys.path.insert(0, 'ocean-simulation_amd'); sys.path.insert(0, 'oracle')
import numpy as np, torch, ocean_hip as oh, oracle as O
for n in (16, 32, 64, 128, 256, 512, 1024):
    for C in (1, 4):
        cas = O.SCENE_CASCADES[:C]
        noise = O.generate_noise(n, 1)
        ctx = oh.OceanContext(n, C, 1, 0); ctx.set_params(O.scene_params(), cas); ctx.set_noise(0, noise); ctx.init_spectrum()
        ctx.step(0.5)
        d, dv, tb = O.OracleOcean(n, O.scene_params(), cas, noise).step(0.5)
        g = ctx.read_all(oh.TEX_DISP); gd = ctx.read_all(oh.TEX_DERIV); gt = ctx.read_all(oh.TEX_TURB)
        print(n, C, 'disp', [round(O.rel_err(g[..., k], d[..., k]), 7) for k in range(3)],
              'deriv', [round(O.rel_err(gd[..., k], dv[..., k]), 7) for k in range(4)], 'turb', round(O.rel_err(gt[..., 0], tb[..., 0]), 7), flush=True)
        ctx.close()
