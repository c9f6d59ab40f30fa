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


def _mips(ctx, tex, C):
    n = ctx.n
    levels = n.bit_length() - 1
    return [[ctx.read_mip(tex, lv, 0, c) for lv in range(1, levels + 1)] for c in range(C)]


@pytest.mark.parametrize("n,ncasc,flags", [(64, 1, 0), (256, 4, 0), (1024, 4, 0),
                                           (256, 3, oh.F_DISPLACEMENT_ONLY), (128, 2, oh.F_MIPS)])
def test_sample_world_matches_restatement(n, ncasc, flags):
    """Bit-exact against the fp32 restatement applied to the context's own textures (the same
    operations in the same order), and within 1e-5 norm-relative per channel against the
    restatement applied to the oracle's textures (DISP/DERIV/TURB parity carried through)."""
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
        for row in range(3):
            for ch in range(4 if row else 3):
                if not full and row == 2:
                    continue
                e = O.rel_err(got[:, row, ch], ref[:, row, ch])
                assert e <= 2e-5, f"row {row} channel {ch}: {e:.2e}"
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
    np.testing.assert_allclose(ctx.sample_world(shifted), got, rtol=0, atol=2e-5)
    with pytest.raises(oh.OceanError) as e:
        ctx.sample_world(pts, tile=1)
    assert e.value.code == oh.E_INVALID_ARG
    assert ctx.sample_world(np.zeros((0, 3), np.float32)).shape == (0, 3, 4)
    ctx.close()
