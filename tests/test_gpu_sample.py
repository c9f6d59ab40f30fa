"""GPU tests of ocean_sample_world: the cascade-summed world sampling of the reference's
consumer (Water.shader:314-348), against the fp32 restatement oracle.sample_world."""
import numpy as np
import pytest

import ocean_hip as oh
import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("require_gpu")]


def _points(m, n, seed, lod_max=0.0, span=5000.0):
    rng = np.random.default_rng(seed)
    p = np.empty((m, 3), np.float32)
    p[:, 0] = rng.uniform(-span, span, m)
    p[:, 1] = rng.uniform(-span, span, m)
    p[:, 2] = rng.uniform(0.0, lod_max, m) if lod_max > 0 else 0.0
    # exact texel centres and edges, negative coordinates, far-away points
    L = O.SCENE_CASCADES[0]["wavelength"]
    p[:4, :2] = [[0.0, 0.0], [L * 0.5 / n, L * 0.5 / n], [-L, 3 * L], [1.0e6, -2.5e6]]
    return p


EPS32 = float(np.finfo(np.float32).eps)


def _sum_bound(gpu, ora, ch):
    """Derived bound on a cascade-summed sample of channel `ch` (ocean.h ocean_sample_world).
    Each cascade's texel differs from the oracle's by at most e_c = max|gpu_c - ora_c|, asserted
    here to be <= 1e-5 max|ora_c| (north_star's tolerance, per cascade and channel). A bilinear or
    trilinear tap is a convex combination, so it moves by at most e_c; the sum over cascades by at
    most sum_c e_c; saturate() is 1-Lipschitz. Slack: a few fp32 roundings of the taps and sums."""
    e = 0.0
    mag = 0.0
    for c in range(gpu.shape[0]):
        d = float(np.abs(gpu[c, ..., ch].astype(np.float64) - ora[c, ..., ch]).max())
        m = float(np.abs(ora[c, ..., ch]).max())
        assert d <= 1e-5 * m + 1e-30, f"texture cascade {c} channel {ch}: {d:.3e} > 1e-5 x {m:.3e}"
        e += d
        mag += m
    return e + 8 * EPS32 * mag


def check_sample_bound(got, ref, disp, deriv, turb):
    """got (GPU sampling of the GPU textures) against ref (the same restatement over the oracle's
    textures): every sampled channel within the derived bound of _sum_bound, and the normal within
    its first-order propagation of the derivative bounds through s = (d.x / (1 + d.z), d.y / (1 +
    d.w)) and n = normalize(-s.x, 1, -s.y) (|dn/ds_k| <= 1 / |(-s.x, 1, -s.y)|)."""
    g, r = got.astype(np.float64), ref.astype(np.float64)
    for ch in range(3):
        b = _sum_bound(disp[0], disp[1], ch)
        assert np.abs(g[:, 0, ch] - r[:, 0, ch]).max() <= b, f"disp channel {ch}"
    if turb is None:
        return
    b = _sum_bound(turb[0], turb[1], 0)
    assert np.abs(g[:, 0, 3] - r[:, 0, 3]).max() <= b + 8 * EPS32 * np.abs(r[:, 0, 3]).max(), "turbulence"
    bd = [_sum_bound(deriv[0], deriv[1], ch) for ch in range(4)]
    for ch in range(4):
        assert np.abs(g[:, 1, ch] - r[:, 1, ch]).max() <= bd[ch], f"deriv channel {ch}"
    d = r[:, 1]
    den_x, den_z = np.abs(1.0 + d[:, 2]), np.abs(1.0 + d[:, 3])
    ok = (den_x > 10 * bd[2]) & (den_z > 10 * bd[3])  # first order holds away from 1 + Dxx ~ 0
    sx, sz = d[:, 0] / (1.0 + d[:, 2]), d[:, 1] / (1.0 + d[:, 3])
    dsx = bd[0] / den_x + np.abs(d[:, 0]) * bd[2] / den_x ** 2
    dsz = bd[1] / den_z + np.abs(d[:, 1]) * bd[3] / den_z ** 2
    nb = 1.05 * (dsx + dsz) / np.sqrt(sx * sx + 1.0 + sz * sz) + 16 * EPS32
    dn = np.abs(g[:, 2, :3] - r[:, 2, :3]).max(axis=1)
    assert ok.mean() > 0.99
    bad = ok & (dn > nb)
    assert not bad.any(), f"normal off its bound at {np.flatnonzero(bad)[:5]}: {dn[bad][:5]} > {nb[bad][:5]}"


def _mips(ctx, tex, C):
    n = ctx.n
    levels = n.bit_length() - 1
    return [[ctx.read_mip(tex, lv, 0, c) for lv in range(1, levels + 1)] for c in range(C)]


@pytest.mark.parametrize("n,ncasc,flags", [(64, 1, 0), (256, 4, 0), (1024, 4, 0),
                                           (256, 3, oh.F_DISPLACEMENT_ONLY), (128, 2, oh.F_MIPS)])
def test_sample_world_matches_restatement(n, ncasc, flags):
    """Bit-exact against the fp32 restatement applied to the context's own textures (the same
    operations in the same order), and against the restatement applied to the oracle's textures
    within the bound derived from the textures' 1e-5 parity (check_sample_bound: a tap is a
    convex combination, the cascade sum adds the per-cascade bounds, the normal propagates the
    derivative bounds to first order)."""
    cas = O.SCENE_CASCADES[:ncasc]
    ctx = oh.OceanContext(n, ncasc, 1, flags)
    ctx.set_params(O.scene_params(), cas)
    noise = O.generate_noise(n, 20251121)
    ctx.set_noise(0, noise)
    ctx.init_spectrum()
    mips = bool(flags & oh.F_MIPS)
    pts = _points(4096, n, n + ncasc, lod_max=(n.bit_length() + 1.0) if mips else 3.0)
    full = not flags & oh.F_DISPLACEMENT_ONLY
    oc = O.OracleOcean(n, O.scene_params(), cas, noise, nplanes=4 if full else 2)
    for t in (0.5, 1.0):
        ctx.step(t)
        disp, deriv, turb = oc.step(t)
    got = ctx.sample_world(pts)
    lengths = [c["wavelength"] for c in cas]
    g_disp = ctx.read_all(oh.TEX_DISP)
    g_deriv = ctx.read_all(oh.TEX_DERIV) if full else None
    g_turb = ctx.read_all(oh.TEX_TURB) if full else None
    want = O.sample_world(g_disp, g_deriv, g_turb, lengths, pts,
                          _mips(ctx, oh.TEX_DERIV, ncasc) if mips else None,
                          _mips(ctx, oh.TEX_TURB, ncasc) if mips else None)
    np.testing.assert_array_equal(got, want)
    if not full:
        assert not got[:, 1].any() and not got[:, 0, 3].any()
    if not mips:  # the oracle's textures (its mip chains are not restated)
        ref = O.sample_world(disp, deriv if full else None, turb if full else None, lengths, pts)
        check_sample_bound(got, ref, (g_disp, disp), (g_deriv, deriv) if full else None,
                           (g_turb, turb) if full else None)
    ctx.close()


def test_sample_world_texel_centres_and_wrap():
    """Known answers: at uv on a texel centre of cascade 0 (one cascade) the sample IS that texel,
    and the Repeat wrap makes x and x + L sample the same values."""
    n, L = 64, 100.0
    cas = [dict(wavelength=L, cutoff_low=1e-4, cutoff_high=1e4, swell=0.3, fade=0.1)]
    ctx = oh.OceanContext(n, 1, 1)
    ctx.set_params(O.scene_params(), cas)
    ctx.generate_noise(3)
    ctx.init_spectrum()
    ctx.step(2.0)
    disp, deriv = ctx.read(oh.TEX_DISP), ctx.read(oh.TEX_DERIV)
    xs, ys = np.meshgrid(np.arange(0, n, 7), np.arange(0, n, 5), indexing="xy")
    pts = np.zeros((xs.size, 3), np.float32)
    pts[:, 0] = (xs.ravel() + 0.5) * L / n
    pts[:, 1] = (ys.ravel() + 0.5) * L / n
    got = ctx.sample_world(pts)
    np.testing.assert_allclose(got[:, 0, :3], disp[ys.ravel(), xs.ravel(), :3], rtol=0, atol=1e-6)
    np.testing.assert_allclose(got[:, 1], deriv[ys.ravel(), xs.ravel()], rtol=0, atol=1e-6)
    shifted = pts.copy()
    shifted[:, 0] += L
    shifted[:, 1] -= 2 * L
    # x + L is a different fp32 coordinate: uv = x / L and the bilinear weight round differently
    # (|du| ~ 2^-24 |x| / L texels), so the wrapped sample agrees to that rounding, not bit for bit
    np.testing.assert_allclose(ctx.sample_world(shifted), got, rtol=0, atol=2e-5)
    with pytest.raises(oh.OceanError) as e:
        ctx.sample_world(pts, tile=1)
    assert e.value.code == oh.E_INVALID_ARG
    assert ctx.sample_world(np.zeros((0, 3), np.float32)).shape == (0, 3, 4)
    ctx.close()


def test_sample_world_state_and_alignment():
    """ocean_sample_world before ocean_init_spectrum is a state error (the cascade wavelengths it
    divides by are not set yet), and the device entry rejects points not 4-byte aligned and out
    not 16-byte aligned instead of faulting on a misaligned float4 store (ocean.h)."""
    import ctypes
    import torch
    ctx = oh.OceanContext(64, 2, 1)
    pts = np.zeros((8, 3), np.float32)
    with pytest.raises(oh.OceanError) as e:
        ctx.sample_world(pts)
    assert e.value.code == oh.E_STATE
    ctx.set_params(O.scene_params(), O.SCENE_CASCADES[:2])
    ctx.generate_noise(5)
    ctx.init_spectrum()
    ctx.step(1.0)
    dev = torch.device("cuda", ctx.device)
    p = torch.zeros(8 * 3 + 1, dtype=torch.float32, device=dev)
    o = torch.zeros(8 * 12 + 4, dtype=torch.float32, device=dev)
    lib, h = ctx.lib, ctx._h
    torch.cuda.synchronize()
    assert lib.ocean_sample_world_device(h, 0, ctypes.c_void_p(p.data_ptr()), 8, ctypes.c_void_p(o.data_ptr())) == oh.OK
    assert lib.ocean_sample_world_device(h, 0, ctypes.c_void_p(p.data_ptr() + 2), 8,
                                         ctypes.c_void_p(o.data_ptr())) == oh.E_INVALID_ARG
    assert lib.ocean_sample_world_device(h, 0, ctypes.c_void_p(p.data_ptr()), 8,
                                         ctypes.c_void_p(o.data_ptr() + 4)) == oh.E_INVALID_ARG
    ctx.synchronize()
    want = ctx.sample_world(pts)
    np.testing.assert_array_equal(o[:96].cpu().numpy().reshape(8, 3, 4), want)
    ctx.close()
