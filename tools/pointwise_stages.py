#!/usr/bin/env python3
"""Where the height channel's pointwise excess comes from, stage by stage, at cfg2
(512^2 x 1, displacement only: pass A8 / B8, the reference's own plane pairing) and cfg3 (4 x 1024^2: the
three-plane pass AQ / BQ).  All figures are SURVEY section 7 clause 2's pointwise error,
max |a - b| / |b| over |b| >= 1e-3 max|b|, worst over frames and cascades, per output channel:

  init      the library's h0 against the oracle's: pointwise, and the share of texels that are bit-identical
            (the init kernel's powf / expf / tanhf / coshf / atan2f / cosf are the device's, the oracle's glibc's)
  frame     the fused frame.  x64o = float64 fed the ORACLE's h0 (what tests/test_gpu_parity.py's bound uses),
            x64l = float64 fed the LIBRARY's own h0.  Pairs: hip-x64o, hip-x64l, oracle-x64o, x64l-x64o (the
            h0 difference carried through exact arithmetic), hip-oracle
  evolve    the unfused evolve with the oracle's h0 uploaded (ocean_write H0) against the oracle's evolve,
            and both against the float64 evolve of the same fp32 h0
  operator  ocean_ifft2d on the oracle's evolved planes against the oracle's radix-2 IFFT, and both against
            numpy's float64 ifft2 of the same fp32 planes

Run once per library / option variant (OCEAN_HIP_LIB, OCEAN_Q select it; the label names it):
    python tools/pointwise_stages.py LABEL out.json [cfg2,cfg3] [init,frame,evolve,operator]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ocean-simulation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402,F401
import ocean_hip as oh  # noqa: E402
import oracle as O  # noqa: E402

FRAC = 1e-3
CONFIGS = {"cfg2": (512, 1, oh.F_DISPLACEMENT_ONLY), "cfg3": (1024, 4, 0)}
TIMES = (0.0, 1 / 60, 100.0)


def pw(a, b):
    return O.pointwise_err(a, b, FRAC)[0]


def ulps(a, b):
    ia = a.astype(np.float32).view(np.int32).astype(np.int64)
    ib = b.astype(np.float32).view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = np.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return np.abs(ia - ib)


def keep_worst(acc, key, vals):
    cur = acc.setdefault(key, {})
    for k, v in vals.items():
        cur[k] = max(cur.get(k, 0.0), v)


def f64_outputs(h0, waves, t, foam_prev, full):
    P = [O.ref64.ifft2d(q) for q in O.ref64.evolve(h0.astype(np.float64), waves.astype(np.float64), t)[:4 if full else 2]]
    out = {"disp": np.stack([P[0].real, P[1].real, P[0].imag], -1)}
    foam = None
    if full:
        out["deriv"] = np.stack([P[2].real, P[2].imag, P[3].real, P[3].imag], -1)
        jac = (1 + P[3].real) * (1 + P[3].imag) - P[1].imag ** 2
        foam = (np.zeros_like(jac) if foam_prev is None else foam_prev) * float(O.FOAM_DECAY)
        foam = np.where(foam < jac, foam + jac, foam)
        out["turb"] = foam[..., None]
    return out, foam


def make(n, C, flags):
    cas = O.SCENE_CASCADES[:C]
    noise = O.generate_noise(n, 20251121)
    ctx = oh.OceanContext(n, C, 1, flags)
    ctx.set_params(O.scene_params(), cas)
    ctx.set_noise(0, noise)
    ctx.init_spectrum()
    return ctx, cas, noise


def row_init(n, C, flags):
    ctx, cas, noise = make(n, C, flags)
    h0o, _ = O.init_spectrum(n, O.scene_params(), cas, noise)
    h0l = ctx.read_all(oh.TEX_H0)
    ctx.close()
    res = {}
    for c in range(C):
        for ch in range(2):
            a, b = h0l[c, ..., ch], h0o[c, ..., ch]
            band = b != 0
            u = ulps(a[band], b[band])
            keep_worst(res, "h0." + "xy"[ch], {"pw": pw(a, b), "norm": O.rel_err(a, b),
                                               "max_ulps": float(u.max()) if u.size else 0.0,
                                               "differ_share": float((u > 0).mean()) if u.size else 0.0})
    return res


def row_frame(n, C, flags):
    full = not flags & oh.F_DISPLACEMENT_ONLY
    ctx, cas, noise = make(n, C, flags)
    h0l = ctx.read_all(oh.TEX_H0)
    oc = O.OracleOcean(n, O.scene_params(), cas, noise, nplanes=4 if full else 2)
    fo, fl = [None] * C, [None] * C
    res, per_t = {}, []
    for t in TIMES:
        ctx.step(t)
        disp, deriv, turb = oc.step(t)
        g = {"disp": ctx.read_all(oh.TEX_DISP)[..., :3]}
        o = {"disp": disp[..., :3]}
        if full:
            g["deriv"], g["turb"] = ctx.read_all(oh.TEX_DERIV), ctx.read_all(oh.TEX_TURB)[..., :1]
            o["deriv"], o["turb"] = deriv, turb[..., :1]
        tw = {}
        for c in range(C):
            xo, fo[c] = f64_outputs(oc.h0[c], oc.waves[c], t, fo[c], full)
            xl, fl[c] = f64_outputs(h0l[c], oc.waves[c], t, fl[c], full)
            for tex in g:
                for ch in range(g[tex].shape[-1]):
                    a, b = g[tex][c, ..., ch], o[tex][c, ..., ch]
                    x_o, x_l = xo[tex][..., ch], xl[tex][..., ch]
                    own = pw(b, x_o)
                    rec = {"hip_x64o": pw(a, x_o), "hip_x64l": pw(a, x_l), "oracle_x64o": own,
                           "x64l_x64o": pw(x_l, x_o), "hip_oracle": pw(a, b)}
                    if own > 0:
                        rec["ratio_test"] = rec["hip_x64o"] / own          # the bound tests/ assert (PW_CEILING)
                        rec["ratio_own_h0"] = rec["hip_x64l"] / own        # each fp32 frame against its own h0
                        rec["ratio_dist"] = rec["hip_oracle"] / own
                    key = f"{tex}.{'xyzw'[ch]}"
                    keep_worst(res, key, rec)
                    keep_worst(tw, key, rec)
        per_t.append({"t": t, "disp.y": tw["disp.y"]})
    ctx.close()
    return res, per_t


def row_evolve(n, C, flags):
    ctx, cas, noise = make(n, C, flags | oh.F_UNFUSED)
    h0o, waves = O.init_spectrum(n, O.scene_params(), cas, noise)
    for c in range(C):
        ctx.write(oh.TEX_H0, h0o[c], 0, c)
    res = {}
    for t in TIMES:
        ctx.evolve(t)
        po = O.evolve(h0o, waves, t)
        for p in range(2 if flags & oh.F_DISPLACEMENT_ONLY else 4):
            gp = ctx.read_all(oh.TEX_PLANE0 + p)
            for c in range(C):
                x = O.ref64.evolve(h0o[c].astype(np.float64), waves[c].astype(np.float64), t)[p]
                for ch, comp in enumerate((x.real, x.imag)):
                    a, b = gp[c, ..., ch], po[p][c, ..., ch]
                    own = pw(b, comp)
                    rec = {"hip_oracle": pw(a, b), "hip_x64": pw(a, comp), "oracle_x64": own}
                    if own > 0:
                        rec["ratio"] = rec["hip_x64"] / own
                    keep_worst(res, f"P{p + 1}.{'re' if ch == 0 else 'im'}", rec)
    ctx.close()
    return res


def row_operator(n, C, flags):
    ctx, cas, noise = make(n, C, (flags & ~oh.F_DISPLACEMENT_ONLY) | oh.F_UNFUSED)
    h0o, waves = O.init_spectrum(n, O.scene_params(), cas, noise)
    res = {}
    for t in TIMES:
        po = O.evolve(h0o, waves, t)
        for p in range(4):
            for c in range(C):
                ctx.write(oh.TEX_PLANE0 + p, po[p][c], 0, c)
        ctx.ifft2d(0b1111)
        for p in range(4):
            gp = ctx.read_all(oh.TEX_PLANE0 + p)
            op = O.ifft2d(po[p])
            for c in range(C):
                x = O.ref64.ifft2d(po[p][c, ..., 0].astype(np.float64) + 1j * po[p][c, ..., 1].astype(np.float64))
                for ch, comp in enumerate((x.real, x.imag)):
                    a, b = gp[c, ..., ch], op[c, ..., ch]
                    own = pw(b, comp)
                    rec = {"hip_oracle": pw(a, b), "hip_x64": pw(a, comp), "oracle_x64": own,
                           "hip_x64_norm": O.rel_err(a, comp), "oracle_x64_norm": O.rel_err(b, comp)}
                    if own > 0:
                        rec["ratio"] = rec["hip_x64"] / own
                    keep_worst(res, f"T[P{p + 1}].{'re' if ch == 0 else 'im'}", rec)
    ctx.close()
    return res


if __name__ == "__main__":
    label, out = sys.argv[1], sys.argv[2]
    cfgs = sys.argv[3].split(",") if len(sys.argv) > 3 else list(CONFIGS)
    rows = sys.argv[4].split(",") if len(sys.argv) > 4 else ["init", "frame", "evolve", "operator"]
    rec = {"label": label, "lib": oh.LIB_PATH, "env": {k: v for k, v in os.environ.items() if k.startswith("OCEAN_")},
           "frac": FRAC, "times": TIMES, "configs": {}}
    for name in cfgs:
        n, C, flags = CONFIGS[name]
        r = rec["configs"][name] = {}
        for row in rows:
            t0 = time.time()
            if row == "init":
                r["init"] = row_init(n, C, flags)
            elif row == "frame":
                r["frame"], r["frame_dy_per_t"] = row_frame(n, C, flags)
            elif row == "evolve":
                r["evolve"] = row_evolve(n, C, flags)
            elif row == "operator":
                r["operator"] = row_operator(n, C, flags)
            print(json.dumps({"label": label, "config": name, "row": row, "s": round(time.time() - t0, 1),
                              "disp.y" if row == "frame" else "first": (r[row].get("disp.y") if row == "frame"
                                                                        else next(iter(r[row].items())))}), flush=True)
            json.dump(rec, open(out, "w"), indent=1)
