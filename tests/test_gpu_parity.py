"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle.

Tolerance: every output channel of every cascade within
norm-relative error max|gpu - oracle| / max|oracle| <= 1e-5 (north_star: "fp32
outputs within 1e-5 relative"); integer-exact quantities (noise, wave numbers,
omega) bit-exact.  Run with `python -m pytest tests -m gpu` on an MI355X.
"""
import ctypes
import json
import os

import numpy as np
import pytest

import ocean_hip as oh
import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("require_gpu")]

TOL = 1e-5
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cplx(a):
    return a[..., 0].astype(np.float64) + 1j * a[..., 1].astype(np.float64)


def make_ctx(n, cascades, params=None, tiles=1, flags=0, seeds=None):
    ctx = oh.OceanContext(n, len(cascades), tiles, flags)
    ctx.set_params(params or O.scene_params(), cascades)
    noises = []
    for t in range(tiles):
        nz = O.generate_noise(n, (seeds or [20251121 + k for k in range(tiles)])[t])
        ctx.set_noise(t, nz)
        noises.append(nz)
    ctx.init_spectrum()
    return ctx, noises


def assert_channels(gpu, ref, tol=TOL, what=""):
    """gpu/ref [C][N][N][ch]: norm-relative error per cascade per channel."""
    for c in range(ref.shape[0]):
        for ch in range(ref.shape[-1]):
            e = O.rel_err(gpu[c, ..., ch], ref[c, ..., ch])
            assert e <= tol, f"{what} cascade {c} channel {ch}: rel err {e:.3e} > {tol}"


# ------------------------------------------------------------------ init
def test_generated_noise_bit_exact():
    ctx = oh.OceanContext(64, 1, 3)
    ctx.generate_noise(777)
    for t in range(3):
        np.testing.assert_array_equal(ctx.read(oh.TEX_NOISE, t), O.generate_noise(64, 777 + t))
    ctx.close()


@pytest.mark.parametrize("shallow", [False, True])
@pytest.mark.parametrize("n", [16, 128, 512])
def test_init_spectrum(n, shallow):
    ctx, (noise,) = make_ctx(n, O.SCENE_CASCADES, O.scene_params(shallow))
    h0, waves = O.init_spectrum(n, O.scene_params(shallow), O.SCENE_CASCADES, noise)
    g_h0, g_w = ctx.read_all(oh.TEX_H0), ctx.read_all(oh.TEX_WAVES)
    # kx, kz, 1/|k| and omega use only correctly rounded + - * / sqrt: bit-exact
    np.testing.assert_array_equal(g_w, waves)
    # h0: every transcendental correctly rounded on both sides (spectrum.hip sp_*, ocean_oracle.c cr_*), the
    # fp32 arithmetic between them in the same order: bit-exact too, conjugate partner .zw included
    np.testing.assert_array_equal(g_h0, h0)
    ctx.close()


# ------------------------------------------------------------ operators
@pytest.mark.parametrize("t", [0.0, 1.25, 100.0])
def test_evolve_operator(t):
    n = 64
    ctx, (noise,) = make_ctx(n, O.SCENE_CASCADES)
    h0, waves = O.init_spectrum(n, O.scene_params(), O.SCENE_CASCADES, noise)
    ctx.evolve(t)
    ref = O.evolve(h0, waves, t)
    for p in range(4):
        got = ctx.read_all(oh.TEX_PLANE0 + p)
        assert_channels(got, ref[p], tol=2e-6, what=f"plane {p}")
    ctx.close()


@pytest.mark.parametrize("n", [16, 32, 64, 128, 256, 512, 1024])
def test_ifft2d_operator_vs_oracle(n):
    """IFFT.InverseFastFourierTransform on random planes vs the reference's radix-2 schedule."""
    C = 2
    ctx = oh.OceanContext(n, C, 1)
    rng = np.random.default_rng(n)
    planes = [rng.standard_normal((C, n, n, 2)).astype(np.float32) for _ in range(4)]
    for p in range(4):
        for c in range(C):
            ctx.write(oh.TEX_PLANE0 + p, planes[p][c], 0, c)
    oh.IFFT(ctx).InverseFastFourierTransform(2)   # plane 2 only
    ctx.ifft2d(0b1001)                             # planes 0 and 3
    for p in range(4):
        got = ctx.read_all(oh.TEX_PLANE0 + p)
        if p == 1:
            np.testing.assert_array_equal(got, planes[p])  # untouched
            continue
        want = O.ifft2d(planes[p])
        assert O.rel_err(cplx(got), cplx(want)) <= TOL
        assert O.rel_err(cplx(got), O.ref64.ifft2d(cplx(planes[p]))) <= 2e-6
    ctx.close()


@pytest.mark.parametrize("n,C,mask", [(2048, 1, 0b0001), (4096, 4, 0b1111), (4096, 1, 0b0110), (4096, 2, 0b1001)])
def test_ifft2d_operator_large_vs_numpy(n, C, mask):
    """The operator at N = 2048 / 4096 on every requested plane of every cascade, against numpy's
    float64 ifft2 (ref64); 4 x 4096^2 x 4 planes is cfg5's whole plane set (2 GiB).  At 4096, in place: rows
    + the decimation-in-frequency fold onto their own rows, then both 2048-point sub-planes of a column
    tile per workgroup (fft2.hip k_rowsf / k_colsf_ip); at 2048 in-place rows, then XCD-paired 8-column
    halves of whole columns (Cols2)."""
    ctx = oh.OceanContext(n, C, 1)
    planes = [p for p in range(4) if mask >> p & 1]

    def slice_data(p, c):
        return np.random.default_rng(1000 * p + c).standard_normal((n, n, 2)).astype(np.float32)

    for p in planes:
        for c in range(C):
            ctx.write(oh.TEX_PLANE0 + p, slice_data(p, c), 0, c)
    ctx.ifft2d(mask)
    for p in range(4):
        for c in range(C):
            got = ctx.read(oh.TEX_PLANE0 + p, 0, c)
            if p not in planes:
                if c == 0 and p == 0:
                    assert not np.any(got), "plane outside the mask written"
                continue
            want = O.ref64.ifft2d(cplx(slice_data(p, c)[None]))[0]
            e = O.rel_err(cplx(got), want)
            assert e <= 2e-6, f"plane {p} cascade {c}: {e:.2e}"
    ctx.close()


@pytest.mark.parametrize("n,chunk_mib", [(2048, None), (2048, 64), (4096, None), (4096, 128), (4096, 768)])
def test_ifft2d_operator_large_vs_oracle(n, chunk_mib, monkeypatch):
    """N = 2048 / 4096 operator against the reference's radix-2 schedule (oracle) on three planes of two
    cascades (6 unit-planes): at 4096 in place, chunks of two unit-planes by default, one at
    OCEAN_OP_CHUNK_MIB=128, all six in one chunk at 768; one chunk at 2048 by default (three at 64);
    plane 3 untouched."""
    if chunk_mib:
        monkeypatch.setenv("OCEAN_OP_CHUNK_MIB", str(chunk_mib))
    C = 2
    O.set_threads(oracle_threads())
    try:
        ctx = oh.OceanContext(n, C, 1)
        rng = np.random.default_rng(7)
        planes = [rng.standard_normal((C, n, n, 2)).astype(np.float32) for _ in range(4)]
        for p in range(4):
            for c in range(C):
                ctx.write(oh.TEX_PLANE0 + p, planes[p][c], 0, c)
        ctx.ifft2d(0b0111)
        np.testing.assert_array_equal(ctx.read_all(oh.TEX_PLANE3), planes[3])
        for p in range(3):
            got = ctx.read_all(oh.TEX_PLANE0 + p)
            want = O.ifft2d(planes[p])
            for c in range(C):
                assert O.rel_err(cplx(got[c]), cplx(want[c])) <= TOL, f"plane {p} cascade {c}"
    finally:
        O.set_threads(1)
    ctx.close()


def test_ifft2d_delta_and_linearity_at_1024():
    """Size-independent properties at the bench size: delta -> plane wave; linearity."""
    n = 1024
    ctx = oh.OceanContext(n, 1, 1)
    d = np.zeros((n, n, 2), np.float32)
    d[7, 300, 0] = 1.0
    ctx.write(oh.TEX_PLANE0, d)
    rng = np.random.default_rng(5)
    a = rng.standard_normal((n, n, 2)).astype(np.float32)
    b = rng.standard_normal((n, n, 2)).astype(np.float32)
    ctx.write(oh.TEX_PLANE1, a)
    ctx.write(oh.TEX_PLANE2, b)
    ctx.write(oh.TEX_PLANE3, (2 * a - b).astype(np.float32))
    ctx.ifft2d(0b1111)
    y, x = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    want = (1 - 2 * ((x + y) % 2)) * np.exp(2j * np.pi * (300 * x + 7 * y) / n)
    assert np.abs(cplx(ctx.read(oh.TEX_PLANE0)) - want).max() < 1e-5
    A, B, L = (cplx(ctx.read(oh.TEX_PLANE0 + p)) for p in (1, 2, 3))
    assert O.rel_err(L, 2 * A - B) < 2e-6
    ctx.close()


def test_fill_operator():
    n = 64
    ctx, _ = make_ctx(n, O.SCENE_CASCADES[:2])
    rng = np.random.default_rng(2)
    planes = [(0.1 * rng.standard_normal((2, n, n, 2))).astype(np.float32) for _ in range(4)]
    turb = np.abs(rng.standard_normal((2, n, n, 4))).astype(np.float32)
    for p in range(4):
        for c in range(2):
            ctx.write(oh.TEX_PLANE0 + p, planes[p][c], 0, c)
    for c in range(2):
        ctx.write(oh.TEX_TURB, turb[c], 0, c)
    ctx.fill()
    disp, deriv, tb = O.fill(planes, turb)
    np.testing.assert_array_equal(ctx.read_all(oh.TEX_DISP), disp)
    np.testing.assert_array_equal(ctx.read_all(oh.TEX_DERIV), deriv)
    np.testing.assert_array_equal(ctx.read_all(oh.TEX_TURB), tb)
    ctx.close()


# ------------------------------------------------------------- full frame
@pytest.mark.parametrize("flags", [0, oh.F_UNFUSED])
def test_golden_fixtures(flags):
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    for case in man["cases"]:
        if case["name"].startswith("ifft"):
            z = np.load(os.path.join(GOLDEN, case["file"]))
            ctx = oh.OceanContext(32, 2, 1, flags)
            for c in range(2):
                ctx.write(oh.TEX_PLANE0, z["input"][c], 0, c)
            ctx.ifft2d(1)
            assert O.rel_err(cplx(ctx.read_all(oh.TEX_PLANE0)), cplx(z["output"])) <= TOL
            ctx.close()
            continue
        z = np.load(os.path.join(GOLDEN, case["file"]))
        n, full = case["n"], case["nplanes"] == 4
        ctx = oh.OceanContext(n, len(case["cascades"]), 1, flags | (0 if full else oh.F_DISPLACEMENT_ONLY))
        ctx.set_params(case["params"], case["cascades"])
        ctx.generate_noise(case["seed"])
        np.testing.assert_array_equal(ctx.read(oh.TEX_NOISE), z["noise"])
        ctx.init_spectrum()
        np.testing.assert_array_equal(ctx.read_all(oh.TEX_H0), z["h0"])  # correctly rounded init: bit-exact
        for f, t in enumerate(case["times"]):
            ctx.step(t)
            assert_channels(ctx.read_all(oh.TEX_DISP)[..., :3], z[f"disp_{f}"][..., :3], what=f"{case['name']} disp {f}")
            if full:
                assert_channels(ctx.read_all(oh.TEX_DERIV), z[f"deriv_{f}"], what=f"{case['name']} deriv {f}")
                assert_channels(ctx.read_all(oh.TEX_TURB), z[f"turb_{f}"], what=f"{case['name']} turb {f}")
        ctx.close()


def oracle_threads():
    """Oracle threads for the full-size cases (the box's CPU share: OMP_NUM_THREADS there)."""
    return int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1))


@pytest.mark.parametrize("n,ncasc,flags", [(256, 1, 0), (256, 2, oh.F_DISPLACEMENT_ONLY),
                                           (512, 1, oh.F_DISPLACEMENT_ONLY), (512, 3, 0),
                                           (1024, 4, 0), (1024, 4, oh.F_UNFUSED), (2048, 1, 0),
                                           (2048, 1, oh.F_UNFUSED), (4096, 1, 0), (4096, 1, oh.F_UNFUSED),
                                           (4096, 1, oh.F_DISPLACEMENT_ONLY), (4096, 4, 0)])
def test_frames_vs_oracle(n, ncasc, flags):
    """BASELINE configs: cfg1-shaped 256^2 x1, cfg2 512^2 displacement only (pass A8 + B8; 256^2: the
    two-plane pass A4 + the side-by-side pass B2D), the scene (512^2 x3),
    cfg3 4 x 1024^2 full outputs, one cfg5 cascade at 4096^2 and cfg5 whole (4 x 4096^2: a 2 GiB
    plane array, 2^31 bytes) through the four-step column passes, against the radix-2 oracle at
    full size; 3 frames (2 for cfg5 whole) so the foam state is exercised.  F_UNFUSED at 2048 / 4096:
    the reference-shaped frame through the operator IFFT's XCD-grouped whole-column tiles."""
    cas = O.SCENE_CASCADES[:ncasc]
    ctx, (noise,) = make_ctx(n, cas, flags=flags)
    nplanes = 2 if flags & oh.F_DISPLACEMENT_ONLY else 4
    O.set_threads(oracle_threads() if n >= 2048 else 1)
    try:
        oc = O.OracleOcean(n, O.scene_params(), cas, noise, nplanes=nplanes)
        times = [0.0, 1.0 / 60.0] if (n == 4096 and ncasc == 4) else [0.0, 1.0 / 60.0, 100.0]
        for f, t in enumerate(times):
            ctx.step(t)
            disp, deriv, turb = oc.step(t)
            assert_channels(ctx.read_all(oh.TEX_DISP)[..., :3], disp[..., :3], what=f"disp f{f}")
            if nplanes == 4:
                assert_channels(ctx.read_all(oh.TEX_DERIV), deriv, what=f"deriv f{f}")
                assert_channels(ctx.read_all(oh.TEX_TURB), turb, what=f"turb f{f}")
            del disp, deriv, turb
    finally:
        O.set_threads(1)
    ctx.close()


# SURVEY.md section 7's second tolerance clause (pointwise 1e-5 where |b| >= 1e-3 max|b|) is infeasible for
# the reference's own algorithm in fp32: on that mask the radix-2 fp32 oracle is 7e-4 .. 1.0e-2 away from
# the float64 frame (tools/pointwise.py, profiles/r06_pointwise/pointwise.json).  This is a
# stated deviation from the spec.  What is asserted instead, per frame, cascade and output channel on the same
# mask, with `own` = the oracle's pointwise error against float64:
#   mine <= PW_CEILING[n][0] * own   the library's pointwise error against float64
#   dist <= PW_CEILING[n][1] * own   its pointwise distance to the oracle
# Since round 6 h0 is bit-exact between the two (correctly rounded init on both sides), so these measure
# the per-frame arithmetic alone.  The ceilings are the measured worst over channels, cascades and frames
# (profiles/r06_pointwise: mine 1.006 / 1.116 / 0.835, dist 1.547 / 1.601 / 1.258 at cfg2 / cfg3 / cfg5)
# plus about 10 %.  dist near sqrt(2) is what two fp32 computations with independent rounding errors of the
# oracle's size give.  (Round 5's single factor 4 covered the init's device-libm h0, then 63-72 % of texels
# a few ulp off: the whole of the 2.5-3.0x excess, tools/pointwise_stages.py.)
PW_FRAC = 1e-3
PW_CEILING = {512: (1.10, 1.70), 1024: (1.25, 1.80), 4096: (1.00, 1.40)}


def _f64_frame(h0, waves, t, foam_prev, full):
    """One cascade's frame in float64 (oracle.ref64's evolve, numpy ifft2, fill, foam) from the oracle's own
    fp32 h0 / wave data: it differs from the oracle only in the per-frame arithmetic."""
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


@pytest.mark.parametrize("n,ncasc,flags,times", [(512, 1, oh.F_DISPLACEMENT_ONLY, (0.0, 1 / 60, 100.0)),
                                                 (1024, 4, 0, (0.0, 1 / 60, 100.0)),
                                                 (4096, 1, 0, (0.0, 1 / 60))])
def test_pointwise_clause(n, ncasc, flags, times):
    """SURVEY section 7 clause 2 as replaced (above): cfg2, cfg3 and one cfg5 cascade, frames with the foam
    carried; clause 1 (1e-5 norm-relative against the oracle) is asserted beside it."""
    full = not flags & oh.F_DISPLACEMENT_ONLY
    cas = O.SCENE_CASCADES[4 - ncasc:] if n == 4096 else O.SCENE_CASCADES[:ncasc]
    ctx, (noise,) = make_ctx(n, cas, flags=flags)
    O.set_threads(oracle_threads() if n >= 2048 else 1)
    try:
        oc = O.OracleOcean(n, O.scene_params(), cas, noise, nplanes=4 if full else 2)
        foam64 = [None] * ncasc
        for t in times:
            ctx.step(t)
            disp, deriv, turb = oc.step(t)
            got = {"disp": ctx.read_all(oh.TEX_DISP)[..., :3]}
            ref = {"disp": disp[..., :3]}
            if full:
                got["deriv"], got["turb"] = ctx.read_all(oh.TEX_DERIV), ctx.read_all(oh.TEX_TURB)[..., :1]
                ref["deriv"], ref["turb"] = deriv, turb[..., :1]
            for c in range(ncasc):
                exact, foam64[c] = _f64_frame(oc.h0[c], oc.waves[c], t, foam64[c], full)
                for tex in got:
                    for ch in range(got[tex].shape[-1]):
                        a, b, x = got[tex][c, ..., ch], ref[tex][c, ..., ch], exact[tex][..., ch]
                        what = f"t={t:g} cascade {c} {tex}.{'xyzw'[ch]}"
                        assert O.rel_err(a, b) <= TOL, what
                        own, _ = O.pointwise_err(b, x, PW_FRAC)
                        mine, _ = O.pointwise_err(a, x, PW_FRAC)
                        dist, _ = O.pointwise_err(a, b, PW_FRAC)
                        fm, fd = PW_CEILING[n]
                        assert mine <= fm * own, f"{what}: pointwise vs float64 {mine:.2e} > {fm} x {own:.2e}"
                        assert dist <= fd * own, f"{what}: pointwise vs oracle {dist:.2e} > {fd} x {own:.2e}"
    finally:
        O.set_threads(1)
        ctx.close()


@pytest.mark.parametrize("n", [1024, 4096])
def test_shallow_frames_vs_oracle(n):
    """Shallow water (depth 4, WaterBody.cs:14's default: the TMA correction's three branches
    and the finite-depth dw/dk, InitialSpectrum.compute:38-43, :87-91) through the fused frame
    at the bench size and at cfg5's N, 2 frames with foam."""
    cas = O.SCENE_CASCADES if n == 1024 else O.SCENE_CASCADES[2:3]
    params = O.scene_params(shallow=True)
    ctx, (noise,) = make_ctx(n, cas, params=params)
    O.set_threads(oracle_threads() if n >= 2048 else 1)
    try:
        oc = O.OracleOcean(n, params, cas, noise)
        for t in (0.75, 1.5):
            ctx.step(t)
            disp, deriv, turb = oc.step(t)
            assert_channels(ctx.read_all(oh.TEX_DISP)[..., :3], disp[..., :3], what=f"disp t={t}")
            assert_channels(ctx.read_all(oh.TEX_DERIV), deriv, what=f"deriv t={t}")
            assert_channels(ctx.read_all(oh.TEX_TURB), turb, what=f"turb t={t}")
    finally:
        O.set_threads(1)
    ctx.close()


@pytest.mark.parametrize("times", [(20000.0, 20000.0 + 1 / 60), (36000.0, 86400.0)])
def test_large_time_vs_oracle(times):
    """cfg3 (4 x 1024^2) at play times of 5.5 h to a day: the phase omega*t passes 2^17 rad
    where sincos_fast hands over from its Cody-Waite path to the library sincosf
    (spectrum_math.h), for the short cascade's high-omega band first (omega up to 14.9 rad/s
    at L = 34, so past t = 8797 s; at 20000 s every texel with omega > 6.55 is past it).  The
    reference computes the fp32 phase omega*t (TimeDependentSpectrum.compute:24-25); the oracle
    runs the same fp32 product through the C library's sinf/cosf."""
    n, cas = 1024, O.SCENE_CASCADES
    ctx, (noise,) = make_ctx(n, cas)
    oc = O.OracleOcean(n, O.scene_params(), cas, noise)
    w = ctx.read_all(oh.TEX_WAVES)
    assert float(w[..., 3].max()) * times[0] > 131072.0  # the hand-over is crossed
    for t in times:
        ctx.step(t)
        disp, deriv, turb = oc.step(t)
        assert_channels(ctx.read_all(oh.TEX_DISP)[..., :3], disp[..., :3], what=f"disp t={t}")
        assert_channels(ctx.read_all(oh.TEX_DERIV), deriv, what=f"deriv t={t}")
        assert_channels(ctx.read_all(oh.TEX_TURB), turb, what=f"turb t={t}")
    ctx.close()


@pytest.mark.parametrize("chunk_mib", [None, 120])
def test_cfg4_shape_chunked_tiles(chunk_mib, monkeypatch):
    """cfg4's per-GPU shard (32 tiles x 4 cascades x 512^2, 128 units) through the three-plane frame
    at the default unit chunking (192 MiB of intermediate at 24 B per texel = 32 units per chunk:
    4 whole chunks) and at OCEAN_CHUNK_MIB=120 (20 units = 5 tiles per chunk: 6 chunks and a partial
    last chunk of 8 units, every chunk rewriting the same reused intermediate region): every tile
    equals a single-tile context bit for bit, and two tiles match the oracle."""
    if chunk_mib is not None:
        monkeypatch.setenv("OCEAN_CHUNK_MIB", str(chunk_mib))
    n, cas, T, seed = 512, O.SCENE_CASCADES, 32, 20251121 + 32
    ctx = oh.OceanContext(n, 4, T)
    ctx.set_params(O.scene_params(), cas)
    ctx.generate_noise(seed)
    ctx.init_spectrum()
    times = (0.25, 0.5)
    for t in times:
        ctx.step(t)
    for tile in range(T):
        single = oh.OceanContext(n, 4, 1)
        single.set_params(O.scene_params(), cas)
        single.generate_noise(seed + tile)
        single.init_spectrum()
        for t in times:
            single.step(t)
        for tex in (oh.TEX_DISP, oh.TEX_DERIV, oh.TEX_TURB):
            np.testing.assert_array_equal(ctx.read_all(tex, tile), single.read_all(tex), err_msg=f"tile {tile}")
        single.close()
    for tile in (5, 31):
        oc = O.OracleOcean(n, O.scene_params(), cas, ctx.read(oh.TEX_NOISE, tile))
        for t in times:
            disp, deriv, turb = oc.step(t)
        assert_channels(ctx.read_all(oh.TEX_DISP, tile)[..., :3], disp[..., :3], what=f"tile {tile} disp")
        assert_channels(ctx.read_all(oh.TEX_DERIV, tile), deriv, what=f"tile {tile} deriv")
        assert_channels(ctx.read_all(oh.TEX_TURB, tile), turb, what=f"tile {tile} turb")
    ctx.close()


@pytest.mark.parametrize("n", [128, 1024])
def test_five_cascades_vs_oracle(n):
    """The ABI's maximum of 5 cascades (ocean.h; Water.shader:139) through the fused frame, a fifth
    short-wave cascade added, against the oracle over 2 frames (foam included)."""
    cas = O.SCENE_CASCADES + [dict(wavelength=9.0, cutoff_low=0.01, cutoff_high=50.0, swell=0.2, fade=0.05)]
    ctx, (noise,) = make_ctx(n, cas)
    oc = O.OracleOcean(n, O.scene_params(), cas, noise)
    for t in (0.0, 2.5):
        ctx.step(t)
        disp, deriv, turb = oc.step(t)
        assert_channels(ctx.read_all(oh.TEX_DISP)[..., :3], disp[..., :3], what=f"N={n} disp t={t}")
        assert_channels(ctx.read_all(oh.TEX_DERIV), deriv, what=f"N={n} deriv t={t}")
        assert_channels(ctx.read_all(oh.TEX_TURB), turb, what=f"N={n} turb t={t}")
    ctx.close()


@pytest.mark.parametrize("n,ncasc,wide", [(256, 4, "32"), (512, 3, "16"), (1024, 1, "8")])
def test_narrow_column_tiles_bit_identical(n, ncasc, wide, monkeypatch):
    """Jobs at N <= 512 with fewer column tiles than CUs run the fused passes on 4-column tiles
    (ocean_create); the frame equals the wide-tile frame bit for bit (OCEAN_TILE_W forces each)."""
    cas = O.SCENE_CASCADES[:ncasc]
    monkeypatch.setenv("OCEAN_TILE_W", "4")
    a, _ = make_ctx(n, cas)
    monkeypatch.setenv("OCEAN_TILE_W", wide)
    b, _ = make_ctx(n, cas)
    for t in (0.5, 1.0):
        a.step(t)
        b.step(t)
    for tex in (oh.TEX_DISP, oh.TEX_DERIV, oh.TEX_TURB):
        np.testing.assert_array_equal(a.read_all(tex), b.read_all(tex))
    a.close()
    b.close()


def test_fused_equals_unfused_to_rounding():
    n, cas = 256, O.SCENE_CASCADES
    a, _ = make_ctx(n, cas)
    b, _ = make_ctx(n, cas, flags=oh.F_UNFUSED)
    for t in (0.3, 0.6):
        a.step(t)
        b.step(t)
    for tex in (oh.TEX_DISP, oh.TEX_DERIV, oh.TEX_TURB):
        assert_channels(a.read_all(tex), b.read_all(tex), tol=1e-6, what=f"tex {tex}")
    a.close()
    b.close()


def test_tiles_are_independent_oceans():
    """cfg4 shape: T tiles, tile k seeded seed+k; each tile equals a single-tile run."""
    n, cas, T = 128, O.SCENE_CASCADES, 3
    ctx = oh.OceanContext(n, 4, T)
    ctx.set_params(O.scene_params(), cas)
    ctx.generate_noise(500)
    ctx.init_spectrum()
    ctx.step(2.0)
    for t in range(T):
        single, _ = make_ctx(n, cas, seeds=[500 + t])
        single.step(2.0)
        for tex in (oh.TEX_DISP, oh.TEX_DERIV, oh.TEX_TURB):
            np.testing.assert_array_equal(ctx.read_all(tex, t), single.read_all(tex))
        single.close()
    ctx.close()


def normal_fp32(deriv):
    """fp32 restatement of normal_from_deriv (spectrum_math.h; Water.shader:346-348 on one
    cascade's derivatives) in the kernel's operation order: every step correctly rounded."""
    d = deriv.astype(np.float32)
    one = np.float32(1.0)
    sx = d[..., 0] / (one + d[..., 2])
    sz = d[..., 1] / (one + d[..., 3])
    inv = one / np.sqrt((sx * sx + one) + sz * sz)
    return np.stack([-sx * inv, inv, -sz * inv, np.zeros_like(inv)], -1)


@pytest.mark.parametrize("n,ncasc,flags", [(128, 2, 0), (128, 2, oh.F_UNFUSED), (1024, 4, 0), (4096, 1, 0)])
def test_normals_derived_output(n, ncasc, flags):
    """NORMAL is normal_from_deriv applied to the context's own DERIV: bit-exact against the
    fp32 restatement; DERIV itself is within 1e-5 of the oracle (as in every frame test), and
    the normal within 1e-5 norm-relative per channel of an fp64 normal of the oracle's DERIV.
    N = 1024 writes it in pass B3's epilogue, N = 4096 in the four-step pass C2's."""
    cas = O.SCENE_CASCADES[:ncasc]
    ctx, (noise,) = make_ctx(n, cas, flags=flags | oh.F_NORMALS)
    ctx.step(0.5)
    got_deriv = ctx.read_all(oh.TEX_DERIV)
    got = ctx.read_all(oh.TEX_NORMAL)
    np.testing.assert_array_equal(got, normal_fp32(got_deriv))
    _, deriv, _ = O.OracleOcean(n, O.scene_params(), cas, noise).step(0.5)
    assert_channels(got_deriv, deriv, what="deriv")
    d = deriv.astype(np.float64)
    sx, sz = d[..., 0] / (1 + d[..., 2]), d[..., 1] / (1 + d[..., 3])
    nrm = np.stack([-sx, np.ones_like(sx), -sz], -1)
    nrm /= np.linalg.norm(nrm, axis=-1, keepdims=True)
    assert_channels(got[..., :3], nrm, what="normal")
    ctx.close()


def test_flat_sea_foam_converges():
    n = 64
    cas = [dict(wavelength=100.0, cutoff_low=1e6, cutoff_high=1e7, swell=0.4, fade=0.1)]
    ctx, _ = make_ctx(n, cas)
    for f in range(40):
        ctx.step(f / 60.0)
    tb = ctx.read(oh.TEX_TURB)
    assert np.all(ctx.read(oh.TEX_DISP)[..., :3] == 0)
    assert abs(float(tb.max()) - 1.0 / (1.0 - np.exp(-2.0))) < 1e-6 and tb.min() == tb.max()
    ctx.close()


def test_foam_state_resume_via_write():
    """Checkpoint/resume: reading TURB after frame k and writing it into a fresh context
    reproduces frame k+1 (the only cross-frame state, ResultTexturesFiller.compute:28-32)."""
    n, cas = 128, O.SCENE_CASCADES[:2]
    a, _ = make_ctx(n, cas)
    a.step(0.1)
    saved = [a.read(oh.TEX_TURB, 0, c) for c in range(2)]
    a.step(0.2)
    b, _ = make_ctx(n, cas)
    for c in range(2):
        b.write(oh.TEX_TURB, saved[c], 0, c)
    b.step(0.2)
    np.testing.assert_array_equal(a.read_all(oh.TEX_TURB), b.read_all(oh.TEX_TURB))
    a.close()
    b.close()


# ----------------------------------------------------------- host mirror
@pytest.mark.parametrize("mode", ["height", "rgba"])
def test_water_body_facade_and_get_water_height(mode):
    """The facade in both readback modes: buoyancyData is the landed slice's .g ([N][N], "height", the
    default) or the whole RGBA slice ("rgba"); GetWaterHeight reads .g either way."""
    def sl(d):
        return d[..., 1] if mode == "height" else d
    wb = oh.scene_water_body(n=256, n_cascades=3, seed=42, readback=mode).Awake()
    wb.Update(1.5)            # steps and requests slice 0 asynchronously (AsyncGPUReadback)
    wb.WaitForReadback()
    disp = wb.DisplacementsTextures()
    assert disp.shape == (3, 256, 256, 4)
    # WaterBody.cs:199-208 mapping: world (x, z) in [-N/2, N/2] -> texel
    for wx, wz in [(0.0, 0.0), (-128.0, -128.0), (127.0, 50.0), (500.0, -500.0)]:
        u = min(max((wx + 128) / 256, 0), 1)
        v = min(max((wz + 128) / 256, 0), 1)
        x, y = min(max(int(u * 256), 0), 255), min(max(int(v * 256), 0), 255)
        assert wb.GetWaterHeight((wx, 0.0, wz)) == disp[0, y, x, 1]
    assert wb.DerivativesTextures().shape == (3, 256, 256, 4) and wb.ctx.read_mip(oh.TEX_DERIV, 8).shape == (1, 1, 4)
    wb.windSpeed = 12.0
    wb.OnValidate()
    wb.Update(1.5)
    wb.Update(1.6)            # a later frame may still find the request in flight: never blocks
    wb.WaitForReadback()
    assert not np.array_equal(wb.DisplacementsTextures(), disp)
    # the landed slice stays in its pinned slot (no copy per frame); buoyancyData is a copy the
    # caller owns, as ToArray() gives: more frames than the ring holds leave a kept copy unchanged
    kept = wb.buoyancyData
    at_16 = sl(wb.ctx.read(oh.TEX_DISP, 0, 0))
    np.testing.assert_array_equal(kept, at_16)
    for k in range(3 * wb.MAX_READBACKS_IN_FLIGHT):
        wb.Update(2.0 + k / 60.0)
    wb.WaitForReadback()
    last = wb.ctx.read(oh.TEX_DISP, 0, 0)
    np.testing.assert_array_equal(wb.buoyancyData, sl(last))
    assert wb.GetWaterHeight((3.0, 0.0, -7.0)) == last[121, 131, 1]  # world (3, -7) -> texel (131, 121)
    assert not np.array_equal(kept, sl(last))
    np.testing.assert_array_equal(kept, at_16)
    wb.OnDisable()
    assert wb.GetWaterHeight((3.0, 0.0, -7.0)) == last[121, 131, 1]  # the slice outlives the ring
    # 16 MiB slices queue faster than they land: the ring fills before the first request completes
    big = oh.scene_water_body(n=1024, n_cascades=1, seed=7, readback=mode).Awake()
    for k in range(3 * big.MAX_READBACKS_IN_FLIGHT):
        big.Update(k / 60.0)
    big.WaitForReadback()
    np.testing.assert_array_equal(big.buoyancyData, sl(big.ctx.read(oh.TEX_DISP, 0, 0)))
    big.OnDisable()


@pytest.mark.parametrize("knob", ["0", "1", "auto"])
def test_disp_cached_knob_bit_identical(knob, monkeypatch):
    """OCEAN_DISP_CACHED (pass BQ's DISP store policy, read at ocean_create) changes no texel: cfg3's frame
    with DISP forced nontemporal, forced default-policy and the automatic choice, against the default."""
    n, cas = 1024, O.SCENE_CASCADES
    ref, _ = make_ctx(n, cas)
    monkeypatch.setenv("OCEAN_DISP_CACHED", knob)
    ctx, _ = make_ctx(n, cas)
    for t in (0.5, 1.0):
        ref.step(t)
        ctx.step(t)
    for tex in (oh.TEX_DISP, oh.TEX_DERIV, oh.TEX_TURB):
        np.testing.assert_array_equal(ctx.read_all(tex), ref.read_all(tex))
    ref.close()
    ctx.close()


def test_height_readback_matches_rgba():
    """ocean_read_height_async is DISP.y of the slice bit for bit, at the same point of the stream as an
    RGBA request (snapshot semantics), for every (tile, cascade); GetWaterHeight of the two facade modes is
    identical over a readback sequence (WaterBody.cs:195-209, :288-296)."""
    n, cas = 256, O.SCENE_CASCADES[:3]
    ctx, _ = make_ctx(n, cas, tiles=2)
    ctx.step(0.5)
    reqs = [(ctx.read_height_async(t, c), ctx.read_async(oh.TEX_DISP, t, c)) for t in range(2) for c in range(3)]
    ctx.step(1.0)  # after the requests: both snapshot the t = 0.5 frame
    for h, rgba in reqs:
        hd, rd = h.data, rgba.data
        assert hd.shape == (n, n) and hd.dtype == np.float32
        np.testing.assert_array_equal(hd, rd[..., 1])
        with pytest.raises(oh.OceanError) as ei:  # untimed (readback timing is off by default)
            h.copy_ms()
        assert ei.value.code == oh.E_STATE
        h.release()
        rgba.release()
    L, out, buf = ctx.lib, ctypes.c_void_p(), oh.PinnedBuffer(n * n * 16)
    for tile, c, nbytes in ((0, 0, n * n * 16), (0, 3, n * n * 4), (2, 0, n * n * 4)):
        assert L.ocean_read_height_async(ctx._h, tile, c, buf.ptr, nbytes, ctypes.byref(out)) == oh.E_INVALID_ARG
    assert L.ocean_read_height_async(ctx._h, 0, 0, None, n * n * 4, ctypes.byref(out)) == oh.E_INVALID_ARG
    buf.release()
    ctx.close()
    bodies = [oh.scene_water_body(n=512, n_cascades=2, seed=9, readback=m).Awake() for m in ("height", "rgba")]
    pts = [(-300.0 + 23.7 * i, 0.0, 280.0 - 31.3 * i) for i in range(24)]
    for f in range(6):
        for wb in bodies:
            wb.Update(f / 60.0)
            wb.WaitForReadback()
        a = [bodies[0].GetWaterHeight(p) for p in pts]
        b = [bodies[1].GetWaterHeight(p) for p in pts]
        assert a == b and any(x != 0.0 for x in a)
        np.testing.assert_array_equal(bodies[0].buoyancyData, bodies[1].buoyancyData[..., 1])
    for wb in bodies:
        wb.OnDisable()


@pytest.mark.parametrize("flags", [oh.F_MIPS, 0, oh.F_UNFUSED])
def test_height_readback_snapshots_behind_later_steps(flags):
    """Snapshot semantics of ocean_read_height_async: each request, made with later steps and an ocean_write of
    DISP queued right behind it, still holds DISP.y of its own frame, bit for bit (DISP depends on t only: a
    second context gives it), with and without the mips, fused and unfused."""
    n, cas = 256, O.SCENE_CASCADES[:2]
    ctx, _ = make_ctx(n, cas, flags=flags)
    ref, _ = make_ctx(n, cas, flags=flags)
    times = [0.1 * k for k in range(8)]
    reqs = []
    for k, t in enumerate(times):
        ctx.step(t)
        reqs.append(ctx.read_height_async(0, k % len(cas)))
        if k == 5:  # DISP overwritten right behind a request
            ctx.write(oh.TEX_DISP, np.zeros((n, n, 4), np.float32), 0, k % len(cas))
    ctx.synchronize()
    for k, (t, rb) in enumerate(zip(times, reqs)):
        ref.step(t)
        np.testing.assert_array_equal(rb.data, ref.read(oh.TEX_DISP, 0, k % len(cas))[..., 1], err_msg=f"frame {k}")
        rb.release()
    ctx.close()
    ref.close()


def test_state_errors():
    ctx = oh.OceanContext(64, 1, 1)
    with pytest.raises(oh.OceanError) as ei:
        ctx.step(0.0)
    assert ei.value.code == oh.E_STATE
    with pytest.raises(oh.OceanError) as ei:
        ctx.init_spectrum()
    assert ei.value.code == oh.E_STATE
    import ctypes
    buf = np.empty(10, np.float32)
    assert ctx.lib.ocean_read(ctx._h, oh.TEX_DISP, 0, 0, buf.ctypes.data, 40) == oh.E_INVALID_ARG
    assert ctx.lib.ocean_read(ctx._h, oh.TEX_DISP, 1, 0, buf.ctypes.data, 64 * 64 * 16) == oh.E_INVALID_ARG
    assert ctx.lib.ocean_read(ctx._h, 99, 0, 0, buf.ctypes.data, 64 * 64 * 16) == oh.E_INVALID_ARG
    ptr, nbytes = ctx.device_ptr(oh.TEX_DISP)
    assert ptr and nbytes == 64 * 64 * 16
    assert ctx.stream() != 0
    d = oh.OceanContext(64, 1, 1, oh.F_DISPLACEMENT_ONLY)
    with pytest.raises(oh.OceanError):
        d.read(oh.TEX_DERIV)
    _ = ctypes
    ctx.close()
    d.close()


def test_kernel_timing_counts_launches():
    ctx, _ = make_ctx(256, O.SCENE_CASCADES)
    ctx.set_kernel_timing(True)
    for f in range(5):
        ctx.step(f / 60)
    ms_a, na = ctx.kernel_stats(0)
    ms_b, nb = ctx.kernel_stats(1)
    assert na == 5 and nb == 5 and ms_a > 0 and ms_b > 0
    ctx.close()


def _ctx_with_env(env, n, cas, **kw):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return make_ctx(n, cas, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("n,flags", [(512, 0), (1024, 0), (512, oh.F_DISPLACEMENT_ONLY),
                                     (256, oh.F_DISPLACEMENT_ONLY)])
def test_mirror_pair_row_pass_bit_identical(n, flags):
    """Pass A4 (rows y and N - y per item, texel pairs k / -k sharing wave data and
    phase) against the per-texel v3 row pass: same arithmetic per texel and per
    butterfly, so every output bit matches (cfg3 / cfg4 shapes, 3 frames incl. foam).  The
    two-plane variant on displacement-only frames (cfg2) within the fp32 tolerance.  Both
    run the four-plane frame (OCEAN_Q=0)."""
    cas = O.SCENE_CASCADES if not flags else O.SCENE_CASCADES[:2]
    a, _ = _ctx_with_env({"OCEAN_A4": "1", "OCEAN_Q": "0"}, n, cas, flags=flags)
    b, _ = _ctx_with_env({"OCEAN_A4": "0", "OCEAN_Q": "0"}, n, cas, flags=flags)
    assert a.step_bytes()[0] < b.step_bytes()[0]  # the row passes differ
    for t in (0.0, 0.5, 250.0):
        a.step(t)
        b.step(t)
    if flags:
        # two planes: the v3 row pass splits N = 16 x ... where A4 runs radix 4 first, so the
        # rounding differs in the last bits (both against the oracle in test_frames_vs_oracle)
        assert_channels(a.read_all(oh.TEX_DISP), b.read_all(oh.TEX_DISP), what="A4 P=2 vs v3")
    else:
        for tex in (oh.TEX_DISP, oh.TEX_DERIV, oh.TEX_TURB):
            np.testing.assert_array_equal(a.read_all(tex), b.read_all(tex))
    a.close()
    b.close()


@pytest.mark.parametrize("n,ncasc,shallow", [(512, 4, False), (1024, 4, False), (1024, 2, True), (4096, 2, False),
                                             (4096, 1, True)])
def test_three_plane_frame_vs_four_plane(n, ncasc, shallow):
    """The three-plane frame (fftq.hip: Q1..Q3 + the Nyquist-line side arrays) against the
    four-plane frame of the reference's planes (OCEAN_Q=0) and against the oracle: the same
    outputs in real arithmetic, so both within the fp32 tolerance, foam over 3 frames
    included.  Scene cascade 0 has nonzero spectrum on the Nyquist lines, where the side
    arrays carry the difference between Q4 and i kz Q1 (without them Dzz is off by ~1e-2).  N = 4096:
    pass A3Q and the four-step column passes forming R[Q4] in C1 (N = 2048 keeps the
    four-plane passes)."""
    O.set_threads(oracle_threads() if n >= 2048 else 1)
    cas = O.SCENE_CASCADES[:ncasc]
    params = O.scene_params(shallow)
    a, noise = _ctx_with_env({"OCEAN_Q": "1"}, n, cas, params=params)
    b, _ = _ctx_with_env({"OCEAN_Q": "0"}, n, cas, params=params)
    assert a.step_bytes()[0] < b.step_bytes()[0]  # the schedules differ
    oc = O.OracleOcean(n, params, cas, noise[0])
    for t in (0.0, 0.5, 250.0):
        a.step(t)
        b.step(t)
        disp, deriv, turb = oc.step(t)
    for tex, ref in ((oh.TEX_DISP, disp[..., :3]), (oh.TEX_DERIV, deriv), (oh.TEX_TURB, turb[..., :1])):
        ga, gb = a.read_all(tex)[..., :ref.shape[-1]], b.read_all(tex)[..., :ref.shape[-1]]
        assert_channels(ga, ref, what=f"Q vs oracle tex {tex}")
        assert_channels(ga, gb, what=f"Q vs four-plane tex {tex}")
    O.set_threads(1)
    a.close()
    b.close()


def test_uploaded_h0_uses_full_h0():
    """After ocean_write(H0) the .zw halves need not be the mirrors' conjugates, so
    the row pass must read h0 itself (pass A4 reads only h0.xy)."""
    n, cas = 1024, O.SCENE_CASCADES[:1]
    a, _ = _ctx_with_env({"OCEAN_A4": "1"}, n, cas)
    b, _ = _ctx_with_env({"OCEAN_A4": "0"}, n, cas)
    h0 = a.read(oh.TEX_H0)
    h0[..., 2:] *= 0.5  # break the conjugate symmetry on purpose
    a.write(oh.TEX_H0, h0)
    b.write(oh.TEX_H0, h0)
    a.step(1.0)
    b.step(1.0)
    for tex in (oh.TEX_DISP, oh.TEX_DERIV):
        np.testing.assert_array_equal(a.read_all(tex), b.read_all(tex))
    a.close()
    b.close()


def test_step_bytes_follows_schedule():
    n, cas = 1024, O.SCENE_CASCADES
    ctx, _ = make_ctx(n, cas)
    tex = n * n * len(cas)
    assert ctx.step_bytes() == (32 * tex, 80 * tex)  # three-plane frame: pass AQ (h0k) + pass BQ
    ctx.write(oh.TEX_H0, ctx.read(oh.TEX_H0))      # uploaded h0: pass A3 reads all of it
    assert ctx.step_bytes() == (48 * tex, 88 * tex)
    ctx.close()
    d, _ = make_ctx(512, cas[:1], flags=oh.F_DISPLACEMENT_ONLY)
    assert d.step_bytes() == (24 * 512 * 512, 32 * 512 * 512)  # two-plane mirror-pair pass A (h0k)
    d.close()


@pytest.mark.parametrize("n", [2048, 4096])
def test_large_n_fused_vs_unfused(n):
    """cfg5 sizes: the fused tile-major passes against the unfused operator chain
    (evolve -> row/column IFFT launches -> fill), 2 frames incl. foam."""
    cas = O.SCENE_CASCADES[:1]
    a, _ = make_ctx(n, cas)
    b, _ = make_ctx(n, cas, flags=oh.F_UNFUSED)
    for t in (0.5, 100.0):
        a.step(t)
        b.step(t)
    for tex in (oh.TEX_DISP, oh.TEX_DERIV, oh.TEX_TURB):
        assert_channels(a.read_all(tex), b.read_all(tex), tol=1e-5, what=f"N={n} tex {tex}")
    a.close()
    b.close()


# ------------------------------------------------------------- mips + readback
def _box_chain(level0):
    """Reference box-filter chain in fp32 with the library's operation order."""
    out, cur = [], level0.astype(np.float32)
    while cur.shape[0] > 1:
        a, b = cur[0::2, 0::2], cur[0::2, 1::2]
        c, d = cur[1::2, 0::2], cur[1::2, 1::2]
        cur = ((a + b) + (c + d)) * np.float32(0.25)
        out.append(cur)
    return out


@pytest.mark.parametrize("n,flags", [(16, 0), (64, 0), (1024, 0), (256, oh.F_UNFUSED), (2048, 0)])
def test_mip_chains_box_filter(n, flags):
    cas = O.SCENE_CASCADES[:2]
    ctx, _ = make_ctx(n, cas, flags=flags | oh.F_MIPS)
    for t in (0.25, 0.5):
        ctx.step(t)
    for tex in (oh.TEX_DERIV, oh.TEX_TURB):
        for c in range(len(cas)):
            chain = _box_chain(ctx.read(tex, 0, c))
            for level, ref in enumerate(chain, start=1):
                np.testing.assert_array_equal(ctx.read_mip(tex, level, 0, c), ref, err_msg=f"tex {tex} level {level}")
    ctx.close()


@pytest.mark.parametrize("n,tiles,flags", [(256, 2, 0), (128, 2, oh.F_UNFUSED), (4096, 1, 0)])
def test_turb_mips_follow_foam_writes_and_resets(n, tiles, flags):
    """TURB's chain after an ocean_write of TURB with unequal channels (foam resume), after ocean_reset_foam, on
    every tile, and at N = 4096 (16-wide foam-state tiles): always the box chain of the TURB texture read back."""
    cas = O.SCENE_CASCADES[:1] if n == 4096 else O.SCENE_CASCADES[:3]
    ctx, _ = make_ctx(n, cas, tiles=tiles, flags=flags | oh.F_MIPS)
    rng = np.random.default_rng(5)

    def check(what):
        for t in range(tiles):
            for c in range(len(cas)):
                turb = ctx.read(oh.TEX_TURB, t, c)
                assert (turb == turb[..., :1]).all(), what  # the fill writes the foam broadcast
                for level, ref in enumerate(_box_chain(turb), start=1):
                    np.testing.assert_array_equal(ctx.read_mip(oh.TEX_TURB, level, t, c), ref,
                                                  err_msg=f"{what} tile {t} cascade {c} level {level}")

    ctx.step(0.25)
    check("first frame")
    for t in range(tiles):
        for c in range(len(cas)):
            ctx.write(oh.TEX_TURB, rng.uniform(-1, 3, (n, n, 4)).astype(np.float32), t, c)
    ctx.step(0.5)
    check("after ocean_write(TURB)")
    ctx.reset_foam()
    ctx.step(0.75)
    check("after ocean_reset_foam")
    ctx.close()


def test_mips_after_many_frames():
    """After 64 frames of 8 slices (2 tiles x 4 cascades at 1024^2; TURB's chain boxed from the foam state,
    csrc/mips.hip) every level of every chain is the box chain of its level 0."""
    ctx, _ = make_ctx(1024, O.SCENE_CASCADES, tiles=2, flags=oh.F_MIPS)
    for f in range(64):
        ctx.step(f / 60.0)
    for tex in (oh.TEX_DERIV, oh.TEX_TURB):
        for t in range(2):
            for c in range(len(O.SCENE_CASCADES)):
                for level, ref in enumerate(_box_chain(ctx.read(tex, t, c)), start=1):
                    np.testing.assert_array_equal(ctx.read_mip(tex, level, t, c), ref,
                                                  err_msg=f"tex {tex} tile {t} cascade {c} level {level}")
    ctx.close()


def test_mip_errors():
    ctx, _ = make_ctx(32, O.SCENE_CASCADES[:1])
    with pytest.raises(oh.OceanError) as e:
        ctx.read_mip(oh.TEX_DERIV, 1)
    assert e.value.code == oh.E_STATE
    ctx.close()
    m, _ = make_ctx(32, O.SCENE_CASCADES[:1], flags=oh.F_MIPS)
    with pytest.raises(oh.OceanError):
        m.read_mip(oh.TEX_DISP, 1)
    with pytest.raises(oh.OceanError):
        m.read_mip(oh.TEX_DERIV, 6)
    m.close()
    with pytest.raises(oh.OceanError) as e:
        oh.OceanContext(32, 1, 1, oh.F_MIPS | oh.F_DISPLACEMENT_ONLY)
    assert e.value.code == oh.E_INVALID_ARG


def test_async_readback_matches_read():
    n, cas = 256, O.SCENE_CASCADES
    ctx, _ = make_ctx(n, cas)
    ctx.step(0.5)
    ctx.set_readback_timing(True)  # ocean_readback_copy_ms needs timed requests (ABI 4)
    reqs = [ctx.read_async(oh.TEX_DISP, 0, c) for c in range(len(cas))]
    reqs.append(ctx.read_async(oh.TEX_TURB, 0, 1))
    ctx.step(1.0)  # after the requests: they snapshot the t = 0.5 frame
    for c in range(len(cas)):
        got = reqs[c].data
        assert reqs[c].done()
        # the copy's own duration (ocean_readback_copy_ms): a 1 MiB device-to-host copy, well under a second
        assert 0.0 < reqs[c].copy_ms() < 1000.0
        reqs[c].release()
        ref = make_ctx(n, cas)[0]
        ref.step(0.5)
        np.testing.assert_array_equal(got, ref.read(oh.TEX_DISP, 0, c))
        ref.close()
    reqs[-1].release()
    ctx.close()


def test_device_noise_matches_restatement():
    n, T = 128, 3
    ctx = oh.OceanContext(n, 1, T)
    ctx.generate_noise_device(99)
    ref = O.generate_noise_device(n, T, 99)
    for t in range(T):
        got = ctx.read(oh.TEX_NOISE, t)
        assert np.abs(got - ref[t]).max() <= 1e-5  # logf ulp differences only; rejection path identical
    g = ctx.read(oh.TEX_NOISE, 0).ravel().astype(np.float64)
    assert abs(g.mean()) < 0.02 and abs(g.var() - 1.0) < 0.03
    ctx.set_params(O.scene_params(), O.SCENE_CASCADES[:1])
    ctx.init_spectrum()  # noise counts as set for every tile
    ctx.step(0.1)
    ctx.close()


def test_whole_frame_intermediate_past_4gib():
    """OCEAN_CHUNK_MIB=0 (one chunk over every unit) on 43 tiles x 4 cascades x 1024^2: the three-plane
    intermediate is 172 units x 24 MiB > 4 GiB, past the 32-bit store offsets of pass AQ, which then
    takes its 64-bit form (fftq.hip go_aq).  Tiles 0 and 42 equal single-tile contexts (the
    32-bit form) bit for bit over two frames."""
    n, cas, T, seed = 1024, O.SCENE_CASCADES, 43, 20251121
    os.environ["OCEAN_CHUNK_MIB"] = "0"  # read once, in ocean_create
    try:
        big = oh.OceanContext(n, 4, T)
    finally:
        os.environ.pop("OCEAN_CHUNK_MIB", None)
    big.set_params(O.scene_params(), cas)
    big.generate_noise_device(seed)
    big.init_spectrum()
    times = (0.5, 1.0)
    for t in times:
        big.step(t)
    for tile in (0, T - 1):
        single = oh.OceanContext(n, 4, 1)
        single.set_params(O.scene_params(), cas)
        single.set_noise(0, big.read(oh.TEX_NOISE, tile))
        single.init_spectrum()
        for t in times:
            single.step(t)
        for tex in (oh.TEX_DISP, oh.TEX_DERIV, oh.TEX_TURB):
            np.testing.assert_array_equal(big.read_all(tex, tile), single.read_all(tex), err_msg=f"tile {tile}")
        single.close()
    big.close()


def test_chunked_frame_equals_whole_frame():
    """Many units: pass A / pass B run per unit chunk (Infinity-Cache-sized); results equal
    the single-launch frame bit for bit."""
    n, cas, T = 128, O.SCENE_CASCADES, 6
    a = _ctx_with_env({"OCEAN_CHUNK_MIB": "1"}, n, cas, tiles=T)[0]   # 2 MiB per unit -> chunks of C units
    b = _ctx_with_env({"OCEAN_CHUNK_MIB": "0"}, n, cas, tiles=T)[0]
    for t in (0.5, 1.0):
        a.step(t)
        b.step(t)
    for tile in range(T):
        for tex in (oh.TEX_DISP, oh.TEX_DERIV, oh.TEX_TURB):
            np.testing.assert_array_equal(a.read_all(tex, tile), b.read_all(tex, tile))
    a.close()
    b.close()


# ------------------------------------------------- cascade subsets + column bands
@pytest.mark.parametrize("n,ncasc,world,flags", [(256, 2, 4, 0), (512, 4, 8, 0), (1024, 4, 8, 0), (4096, 2, 4, 0),
                                                 (4096, 4, 8, 0), (512, 1, 4, oh.F_DISPLACEMENT_ONLY),
                                                 (256, 1, 2, oh.F_DISPLACEMENT_ONLY)])
def test_split_ocean_shards_bit_identical(n, ncasc, world, flags):
    """One ocean split over `world` GPUs by ocean_hip.shard.plan_shard (cascade blocks,
    then column bands: cfg5's 8-GPU split at world = 2 x cascades), each shard its own
    context here on one GPU: every texel of every shard equals the whole ocean's bit for
    bit (the same arithmetic per texel; no data exchange), and columns outside a shard's
    band stay untouched (zero).  N = 512 / 1024 run the mirror-pair row pass, 4096 the
    four-step column passes; (4096, 4, 8) is cfg5's real 8-GPU plan (one cascade, half the
    columns per rank); the displacement-only cases (cfg2's shape) run the two-plane mirror-pair
    row pass and the side-by-side column pass on narrow bands."""
    from ocean_hip.shard import plan_shard
    cas = O.SCENE_CASCADES[:ncasc]
    whole, _ = make_ctx(n, cas, flags=flags)
    shards = []
    for r in range(world):
        sh = plan_shard(1, ncasc, n, world, r, interleave=False)
        ctx, _ = make_ctx(n, cas[sh.casc0:sh.casc0 + sh.cascades], flags=flags)
        ctx.set_column_band(sh.x0, sh.nx)
        shards.append((sh, ctx))
    assert any(sh.nx < n for sh, _ in shards)
    for t in (0.25, 3.0):
        whole.step(t)
        for _, ctx in shards:
            ctx.step(t)
    for tex in ((oh.TEX_DISP,) if flags else (oh.TEX_DISP, oh.TEX_DERIV, oh.TEX_TURB)):
        ref = whole.read_all(tex)
        for sh, ctx in shards:
            got = ctx.read_all(tex)
            band = slice(sh.x0, sh.x0 + sh.nx)
            np.testing.assert_array_equal(got[..., band, :], ref[sh.casc0:sh.casc0 + sh.cascades, :, band, :],
                                          err_msg=f"tex {tex} shard {sh}")
            outside = np.ones(n, bool)
            outside[band] = False
            assert not got[..., outside, :].any(), f"tex {tex} shard {sh} wrote outside its band"
    whole.close()
    for _, ctx in shards:
        ctx.close()


def test_column_parity_shards_vs_oracle():
    """cfg5 on 8 GPUs as plan_shard splits it: 4 cascades x 4096^2, each cascade's even and odd
    columns on two ranks (ocean_set_column_parity: pass A3P folds every row to z_b and transforms
    it at 2048 points), each shard its own context here on one GPU.  Every shard's compact
    textures (column m = x 2m + b) against the oracle's columns b, b + 2, ... at 1e-5 per cascade
    and channel, over two frames (foam included); the texture columns m >= N/2 stay untouched; and
    the shards match the whole single-GPU frame within the same tolerance."""
    from ocean_hip.shard import plan_shard
    n, cas = 4096, O.SCENE_CASCADES
    O.set_threads(min(16, os.cpu_count() or 1))
    whole, (noise,) = make_ctx(n, cas)
    shards = []
    for r in range(8):
        sh = plan_shard(1, 4, n, 8, r)
        assert sh.parity == r % 2 and sh.cascades == 1
        ctx, _ = make_ctx(n, cas[sh.casc0:sh.casc0 + 1])
        ctx.set_column_parity(sh.parity)
        shards.append((sh, ctx))
    oc = O.OracleOcean(n, O.scene_params(), cas, noise)
    for t in (0.25, 3.0):
        whole.step(t)
        for _, ctx in shards:
            ctx.step(t)
        disp, deriv, turb = oc.step(t)
    O.set_threads(1)
    refs = {oh.TEX_DISP: disp[..., :3], oh.TEX_DERIV: deriv, oh.TEX_TURB: turb}
    for tex, ref in refs.items():
        w = whole.read_all(tex)[..., :ref.shape[-1]]
        for sh, ctx in shards:
            got = ctx.read(tex)
            assert not got[:, n // 2:].any(), f"tex {tex} shard {sh}: wrote past the compact half"
            mine = got[None, :, :n // 2, :ref.shape[-1]]
            c, b = sh.casc0, sh.parity
            assert_channels(mine, ref[c:c + 1, :, b::2], what=f"tex {tex} shard {sh} vs oracle")
            assert_channels(mine, w[c:c + 1, :, b::2], what=f"tex {tex} shard {sh} vs whole frame")
    whole.close()
    for _, ctx in shards:
        ctx.close()


def test_column_parity_call_orders():
    """a column parity set BEFORE ocean_init_spectrum (h0k is allocated then, and filled by
    the init), and an H0 upload on a parity context (the frame then refuses, E_STATE) followed by a
    re-init, both give the oracle's columns b, b + 2, ... at 1e-5 (one 4096^2 cascade, two frames)."""
    n, cas = 4096, O.SCENE_CASCADES[3:4]
    noise = O.generate_noise(n, 20251121)
    ctx = oh.OceanContext(n, 1, 1, 0)
    ctx.set_params(O.scene_params(), cas)
    ctx.set_noise(0, noise)
    ctx.set_column_parity(1)
    ctx.init_spectrum()
    O.set_threads(min(16, os.cpu_count() or 1))
    try:
        oc = O.OracleOcean(n, O.scene_params(), cas, noise)

        def check(t, what):
            ctx.step(t)
            disp, deriv, turb = oc.step(t)
            for tex, ref in ((oh.TEX_DISP, disp[..., :3]), (oh.TEX_DERIV, deriv), (oh.TEX_TURB, turb)):
                got = ctx.read(tex)[None, :, :n // 2, :ref.shape[-1]]
                assert_channels(got, ref[:, :, 1::2], what=f"{what} tex {tex}")
        check(0.5, "parity before init")
        h0 = ctx.read(oh.TEX_H0)
        ctx.write(oh.TEX_H0, h0)  # an upload: .zw may no longer be conj h0(-k) as far as the context knows
        with pytest.raises(oh.OceanError) as e:
            ctx.step(0.75)
        assert e.value.code == oh.E_STATE
        ctx.init_spectrum()  # the spectrum (and h0k) again from the parameters
        check(1.0, "re-init after an H0 upload")
    finally:
        O.set_threads(1)
        ctx.close()


def test_column_parity_errors():
    ctx, _ = make_ctx(1024, O.SCENE_CASCADES[:1])
    with pytest.raises(oh.OceanError) as e:
        ctx.set_column_parity(0)
    assert e.value.code == oh.E_UNSUPPORTED
    ctx.close()
    ctx, _ = make_ctx(4096, O.SCENE_CASCADES[:1])
    with pytest.raises(oh.OceanError) as e:
        ctx.set_column_parity(2)
    assert e.value.code == oh.E_INVALID_ARG
    ctx.set_column_parity(1)
    a, b = ctx.step_bytes()
    ctx.set_column_parity(-1)
    assert ctx.step_bytes()[1] > b  # the whole band again
    ctx.set_column_parity(0)
    with pytest.raises(oh.OceanError) as e:
        ctx.sample_world(np.zeros((1, 3), np.float32))
    assert e.value.code == oh.E_UNSUPPORTED
    ctx.set_column_band(0, 4096)  # a band replaces the parity
    ctx.step(0.5)
    ctx.close()


def test_column_band_narrow_and_restored():
    """A 16-column band at an interior offset (N = 1024, tiles of 8), then the whole band
    again: the band context's next frames match the whole-band context everywhere (foam
    of the columns outside the band restarted from its frozen state is not compared)."""
    n, cas = 1024, O.SCENE_CASCADES[:1]
    a, _ = make_ctx(n, cas)
    b, _ = make_ctx(n, cas)
    b.set_column_band(496, 16)
    a.step(0.5)
    b.step(0.5)
    np.testing.assert_array_equal(b.read(oh.TEX_DISP)[:, 496:512], a.read(oh.TEX_DISP)[:, 496:512])
    b.set_column_band(0, n)
    a.step(1.0)
    b.step(1.0)
    np.testing.assert_array_equal(b.read(oh.TEX_DISP), a.read(oh.TEX_DISP))
    np.testing.assert_array_equal(b.read(oh.TEX_DERIV), a.read(oh.TEX_DERIV))
    a.close()
    b.close()


def test_column_band_errors_and_bytes():
    n, cas = 1024, O.SCENE_CASCADES
    ctx, _ = make_ctx(n, cas)
    for x0, nx in ((8, 16), (0, 8), (0, 0), (1024 - 16, 32), (-16, 16)):
        with pytest.raises(oh.OceanError) as e:
            ctx.set_column_band(x0, nx)
        assert e.value.code == oh.E_INVALID_ARG
    tex = n * n * len(cas)
    ctx.set_column_band(512, 512)
    assert ctx.step_bytes() == (8 * tex + 12 * tex, 40 * tex)  # h0k read whole, the rest halves (Q frame)
    ctx.close()
    u, _ = make_ctx(256, cas[:1], flags=oh.F_UNFUSED)
    with pytest.raises(oh.OceanError) as e:
        u.set_column_band(0, 128)
    assert e.value.code == oh.E_UNSUPPORTED
    u.set_column_band(0, 256)  # the whole band is always allowed
    u.close()


@pytest.mark.parametrize("n,bands", [(2048, "4"), (4096, "0")])
def test_four_step_column_bands_bit_identical(n, bands):
    """N >= 2048: the column passes C1 + C2 run per (unit, column band) so that C2 re-reads
    C1's output from the Infinity Cache (OCEAN_C4_BANDS; 0 = auto, 2 bands at 4096).  The
    per-texel arithmetic is unchanged: bit-identical to one launch pair over everything."""
    cas = O.SCENE_CASCADES[:2] if n == 2048 else O.SCENE_CASCADES[:1]
    a, _ = _ctx_with_env({"OCEAN_C4_BANDS": "1"}, n, cas)
    b, _ = _ctx_with_env({"OCEAN_C4_BANDS": bands}, n, cas)
    for t in (0.5, 2.0):
        a.step(t)
        b.step(t)
    for tex in (oh.TEX_DISP, oh.TEX_DERIV, oh.TEX_TURB):
        np.testing.assert_array_equal(a.read_all(tex), b.read_all(tex))
    a.close()
    b.close()


# ------------------------------------------------------------ random scenes
# Every test above uses the scene of Waves.unity (deep or shallow).  These sweep the physical inputs the
# WaterBody / WaterCascade inspector exposes (WaterBody.cs:10-14, WaterCascade.cs:10-24), seeded:
# wind speeds 1-32 m/s, axis-aligned, diagonal, arbitrary and unnormalised wind directions, fetch
# 300 m-1000 km, depth 0.3-5000 m (every TMA branch), gravity 1-25, cascade wavelengths 10-3000 m with cutoffs
# that drop low rings or clip the high band, swell and fade over [0, 1], 1-5 cascades, 1-2 tiles,
# N = 16-1024, full outputs / displacement only / the unfused reference-shaped frame, and times up to
# 5000 s.  Plus the script defaults (WaterBody.cs:10-14 and WaterCascade.cs:10-24: U10 1, wind (1, 1),
# fetch 1, depth 4, N 256; L 10, cutoffs 1e-4 / 5, swell 0.4, fade 0.1), which no scene file uses.
# Checked: noise, wave data and h0 bit-exact; every output channel within the 1e-5 norm-relative tolerance
# over three frames with the foam carried.
_AXES = [(1.0, 0.0), (0.0, 1.0), (-1.0, 0.0), (0.0, -1.0), (1.0, 1.0), (3.0, -4.0)]


def _random_scene(seed):
    r = np.random.default_rng(1000 + seed)
    n = int(r.choice([16, 32, 64, 128, 256, 512, 1024]))
    C = int(r.integers(1, 6))
    flags = int(r.choice([0, 0, oh.F_DISPLACEMENT_ONLY, oh.F_UNFUSED]))
    tiles = int(r.integers(1, 3)) if n <= 256 else 1
    if r.random() < 0.5:
        wx, wy = _AXES[int(r.integers(len(_AXES)))]
    else:
        a = r.uniform(0, 2 * np.pi)
        wx, wy = float(np.cos(a)), float(np.sin(a))
    params = dict(wind_speed=float(10 ** r.uniform(0, 1.5)), wind_dir_x=wx, wind_dir_y=wy,
                  gravity=float(r.choice([9.81, r.uniform(1.0, 25.0)])), fetch=float(10 ** r.uniform(2.5, 6)),
                  depth=float(10 ** r.uniform(-0.5, 3.7)))
    cascades = []
    for _ in range(C):
        L = float(10 ** r.uniform(1, 3.5))
        dk = 2 * np.pi / L
        cascades.append(dict(wavelength=L, cutoff_low=float(dk * 10 ** r.uniform(-3, 0.8)),
                             cutoff_high=float(dk * n / 2 * 10 ** r.uniform(-0.8, 1.0)),
                             swell=float(r.uniform(0, 1)), fade=float(r.uniform(0, 1))))
    times = [0.0, float(r.uniform(0, 50)), float(r.uniform(100, 5000))]
    return n, flags, tiles, params, cascades, times


SCRIPT_DEFAULTS = (256, 0, 1, dict(wind_speed=1.0, wind_dir_x=1.0, wind_dir_y=1.0, gravity=9.81, fetch=1.0, depth=4.0),
                   [dict(wavelength=10.0, cutoff_low=1e-4, cutoff_high=5.0, swell=0.4, fade=0.1)], [0.0, 1 / 60, 100.0])


@pytest.mark.parametrize("case", ["defaults"] + [f"random{s}" for s in range(30)])
def test_scene_sweep_vs_oracle(case):
    n, flags, tiles, params, cascades, times = SCRIPT_DEFAULTS if case == "defaults" else _random_scene(int(case[6:]))
    seeds = [4242 + t for t in range(tiles)]
    ctx, noises = make_ctx(n, cascades, params, tiles=tiles, flags=flags, seeds=seeds)
    nplanes = 2 if flags & oh.F_DISPLACEMENT_ONLY else 4
    what = f"{case}: n {n} C {len(cascades)} tiles {tiles} flags {flags} params {params}"
    O.set_threads(oracle_threads() if n >= 512 else 1)
    try:
        ocs = []
        for t, noise in enumerate(noises):
            h0, waves = O.init_spectrum(n, params, cascades, noise)
            np.testing.assert_array_equal(ctx.read(oh.TEX_NOISE, t), noise, err_msg=what)
            np.testing.assert_array_equal(ctx.read_all(oh.TEX_WAVES, t), waves, err_msg=what)
            np.testing.assert_array_equal(ctx.read_all(oh.TEX_H0, t), h0, err_msg=what)
            ocs.append(O.OracleOcean(n, params, cascades, noise, nplanes=nplanes))
        for f, tm in enumerate(times):
            ctx.step(tm)
            for t, oc in enumerate(ocs):
                disp, deriv, turb = oc.step(tm)
                assert np.isfinite(disp).all(), what
                assert_channels(ctx.read_all(oh.TEX_DISP, t)[..., :3], disp[..., :3], what=f"{what} tile {t} disp f{f}")
                if nplanes == 4:
                    assert_channels(ctx.read_all(oh.TEX_DERIV, t), deriv, what=f"{what} tile {t} deriv f{f}")
                    assert_channels(ctx.read_all(oh.TEX_TURB, t), turb, what=f"{what} tile {t} turb f{f}")
    finally:
        O.set_threads(1)
    ctx.close()
