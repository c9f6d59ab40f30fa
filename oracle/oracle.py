"""ctypes/numpy front end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, as the checker.  The product (ocean-simulation_amd/) never does.

`liboceanoracle.so` is the fp32 C restatement in ocean_oracle.c (reference
file:line citations are there).  `ref64` below is an independent float64 numpy
restatement whose 2D IFFT is numpy.fft (not the reference's butterfly
schedule); it cross-checks the C oracle in tests/test_oracle.py.

Parity status: "parity unpinned" by reference-produced vectors -- the reference
(Unity/HLSL) ships none and cannot run here; see DESIGN.md section 2.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboceanoracle.so")
_lib = None

FOAM_DECAY = np.float32(0.135335283236612691894)


class OrParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in
                ("wind_speed", "wind_dir_x", "wind_dir_y", "gravity", "fetch", "depth")]


class OrCascade(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in
                ("wavelength", "cutoff_low", "cutoff_high", "swell", "fade")]


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "ocean_oracle.c"))):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboceanoracle.so"])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        i, f = ctypes.c_int, ctypes.c_float
        L.oracle_generate_noise.argtypes = [i, ctypes.c_uint64, fp]
        L.oracle_init_spectrum.argtypes = [i, i, ctypes.POINTER(OrParams), ctypes.POINTER(OrCascade), fp, fp, fp]
        L.oracle_conjugate_spectrum.argtypes = [i, i, fp]
        L.oracle_evolve.argtypes = [i, i, fp, fp, f, fp, fp, fp, fp]
        L.oracle_twiddle_table.argtypes = [i, fp]
        L.oracle_ifft2d.argtypes = [i, i, fp, fp, fp]
        L.oracle_fill.argtypes = [i, i, fp, fp, fp, fp, fp, fp, fp]
        L.oracle_step.argtypes = [i, i, i, fp, fp, fp, f, fp, fp, fp, fp, fp]
        L.oracle_set_threads.argtypes = [i]
        for fn in (L.oracle_generate_noise, L.oracle_init_spectrum, L.oracle_conjugate_spectrum, L.oracle_evolve,
                   L.oracle_twiddle_table, L.oracle_ifft2d, L.oracle_fill, L.oracle_step, L.oracle_set_threads):
            fn.restype = None
        _lib = L
    return _lib


def set_threads(n: int) -> None:
    """Threads of the per-frame loops (evolve, IFFT stages, fill); 1 (the default) is the
    scalar restatement.  Results do not depend on it (element-wise stages)."""
    lib().oracle_set_threads(int(n))


def _p(a):
    if a is None:
        return None
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _params(p: dict) -> OrParams:
    return OrParams(p["wind_speed"], p["wind_dir_x"], p["wind_dir_y"], p["gravity"], p["fetch"], p["depth"])


def _cascades(cs) -> ctypes.Array:
    arr = (OrCascade * len(cs))()
    for k, c in enumerate(cs):
        arr[k] = OrCascade(c["wavelength"], c["cutoff_low"], c["cutoff_high"], c["swell"], c["fade"])
    return arr


def generate_noise(n: int, seed: int) -> np.ndarray:
    out = np.empty((n, n, 2), np.float32)
    lib().oracle_generate_noise(n, ctypes.c_uint64(seed), _p(out))
    return out


_G = np.uint64(0x9E3779B97F4A7C15)


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def generate_noise_device(n: int, tiles: int, seed: int) -> np.ndarray:
    """Restatement of the library's on-device noise (ocean.h ocean_generate_noise_device):
    per texel a counter-based uniform stream, each of g1, g2 from the polar loop of
    WaterBody.cs:71-81.  Rejection decisions are exact; g differs from the device only by
    the ulp-level difference of logf.  float32 [tiles][N][N][2]."""
    with np.errstate(over="ignore"):
        texel = np.arange(n * n, dtype=np.uint64)
        out = np.empty((tiles, n * n, 2), np.float32)
        for t in range(tiles):
            key = _mix64(np.uint64(seed) + np.uint64(t) + _G) ^ (texel * np.uint64(0xD1B54A32D192ED03))
            k = np.zeros(n * n, np.uint64)

            def uniform(idx):
                k[idx] += np.uint64(1)
                h = _mix64(key[idx] + k[idx] * _G)
                return (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
            for c in range(2):
                g = np.empty(n * n, np.float32)
                todo = np.arange(n * n)
                while todo.size:
                    v1 = np.float32(2.0) * uniform(todo) - np.float32(1.0)
                    v2 = np.float32(2.0) * uniform(todo) - np.float32(1.0)
                    q = v1 * v1 + v2 * v2
                    ok = (q < np.float32(1.0)) & (q != np.float32(0.0))
                    qa = q[ok]
                    g[todo[ok]] = v1[ok] * np.sqrt(np.float32(-2.0) * np.log(qa) / qa)
                    todo = todo[~ok]
                out[t, :, c] = g
    return out.reshape(tiles, n, n, 2)


def init_spectrum(n, params, cascades, noise, conjugate=True):
    C = len(cascades)
    h0 = np.empty((C, n, n, 4), np.float32)
    waves = np.empty((C, n, n, 4), np.float32)
    noise = np.ascontiguousarray(noise, np.float32)
    lib().oracle_init_spectrum(n, C, ctypes.byref(_params(params)), _cascades(cascades), _p(noise), _p(h0), _p(waves))
    if conjugate:
        lib().oracle_conjugate_spectrum(n, C, _p(h0))
    return h0, waves


def evolve(h0, waves, t):
    C, n = h0.shape[0], h0.shape[1]
    planes = [np.empty((C, n, n, 2), np.float32) for _ in range(4)]
    lib().oracle_evolve(n, C, _p(h0), _p(waves), ctypes.c_float(t), *[_p(q) for q in planes])
    return planes


def twiddle_table(n):
    logn = int(np.log2(n))
    tab = np.empty((logn, n, 4), np.float32)
    lib().oracle_twiddle_table(n, _p(tab))
    return tab


def ifft2d(plane):
    """Reference IFFT (IFFT.cs:66-94) on a float32 [C][N][N][2] array; returns a new array."""
    C, n = plane.shape[0], plane.shape[1]
    out = np.ascontiguousarray(plane, np.float32).copy()
    pp = np.empty_like(out)
    lib().oracle_ifft2d(n, C, _p(twiddle_table(n)), _p(out), _p(pp))
    return out


def fill(planes, turb_prev=None, full=True):
    C, n = planes[0].shape[0], planes[0].shape[1]
    disp = np.empty((C, n, n, 4), np.float32)
    deriv = np.empty((C, n, n, 4), np.float32) if full else None
    turb = (np.zeros((C, n, n, 4), np.float32) if turb_prev is None else turb_prev.copy()) if full else None
    p2 = planes[2] if full else None
    p3 = planes[3] if full else None
    lib().oracle_fill(n, C, _p(planes[0]), _p(planes[1]), _p(p2), _p(p3), _p(disp), _p(deriv), _p(turb))
    return disp, deriv, turb


class OracleOcean:
    """Stateful CPU oracle of one (tile) ocean: mirrors WaterBody's init + per-frame schedule."""

    def __init__(self, n, params, cascades, noise, nplanes=4):
        self.n, self.C, self.nplanes = n, len(cascades), nplanes
        self.h0, self.waves = init_spectrum(n, params, cascades, noise)
        self.table = twiddle_table(n)
        self.planes = np.empty((4, self.C, n, n, 2), np.float32)
        self.pingpong = np.empty((self.C, n, n, 2), np.float32)
        self.disp = np.zeros((self.C, n, n, 4), np.float32)
        self.deriv = np.zeros((self.C, n, n, 4), np.float32)
        self.turb = np.zeros((self.C, n, n, 4), np.float32)

    def step(self, t):
        full = self.nplanes == 4
        lib().oracle_step(self.n, self.C, self.nplanes, _p(self.h0), _p(self.waves), _p(self.table),
                          ctypes.c_float(t), _p(self.planes), _p(self.pingpong), _p(self.disp),
                          _p(self.deriv) if full else None, _p(self.turb) if full else None)
        return self.disp, (self.deriv if full else None), (self.turb if full else None)


# ---------------------------------------------------------------------------
# Independent float64 restatement (numpy.fft for the transform).
# ---------------------------------------------------------------------------
class ref64:
    @staticmethod
    def init_spectrum(n, p, cascades, noise):
        PI = float(np.float32(3.14159265))
        g, U, F, D = p["gravity"], p["wind_speed"], p["fetch"], p["depth"]
        wp = 22.0 * abs(g * g / (U * F)) ** 0.3333
        half = n // 2
        nz, nx = np.meshgrid(np.arange(n) - half, np.arange(n) - half, indexing="ij")
        C = len(cascades)
        h0 = np.zeros((C, n, n, 4))
        waves = np.zeros((C, n, n, 4))
        wd = np.array([p["wind_dir_x"], p["wind_dir_y"]], np.float64)
        wd = wd / np.linalg.norm(wd)
        wtheta = np.arctan2(wd[1], wd[0])
        for c, cs in enumerate(cascades):
            dk = 2.0 * PI / cs["wavelength"]
            kx, kz = nx * dk, nz * dk
            km = np.hypot(kx, kz)
            band = (km >= cs["cutoff_low"]) & (km <= cs["cutoff_high"])
            kms = np.where(band, km, 1.0)
            w = np.sqrt(g * kms)
            wh = w * np.sqrt(D / g)
            tma = np.where(wh <= 1.0, 0.5 * wh * wh, np.where(wh < 2.0, 1.0 - 0.5 * (2.0 - wh) ** 2, 1.0))
            alpha = 0.076 * abs(U * U / (F * g)) ** 0.22
            sigma = np.where(w <= wp, 0.07, 0.09)
            r = np.exp(-((w - wp) ** 2) / (2 * sigma * sigma * wp * wp))
            J = alpha * g * g / w ** 5 * np.exp(-1.25 * (wp / w) ** 4) * 3.3 ** r
            mu = -2.33 - 1.45 * (U / (g / wp) - 1.17)
            sp = np.where(w < 1.05 * wp, 6.97 * np.abs(w / wp) ** 4.06, 9.77 * np.abs(w / wp) ** mu)
            s = sp + 16 * np.tanh(w / wp) * cs["swell"] ** 2
            q = np.where(s <= 0.4,
                         0.09 * s ** 3 + (np.log(2) ** 2 / PI - PI / 12) * s ** 2 + np.log(2) / PI * s + 1 / (2 * PI),
                         np.sqrt(s) / (2 * np.sqrt(PI)) + 1 / (16 * np.sqrt(PI * s)))
            theta = np.arctan2(kz, kx)
            Dsp = q * np.abs(np.cos(0.5 * (theta - wtheta))) ** (2 * s)
            with np.errstate(over="ignore"):
                ch = np.cosh(kms * D)
            dwdk = g * (D * kms / ch / ch + np.tanh(np.minimum(kms * D, 20))) / (2 * w)
            fade = np.exp(-cs["fade"] ** 2 * kms ** 2)
            amp = np.sqrt(2 * tma * J * Dsp * fade * dwdk / kms * dk * dk)
            h0[c, ..., 0] = np.where(band, noise[..., 0] / 2 * amp, 0)
            h0[c, ..., 1] = np.where(band, noise[..., 1] / 2 * amp, 0)
            waves[c, ..., 0] = kx
            waves[c, ..., 1] = np.where(band, 1.0 / kms, 1.0)
            waves[c, ..., 2] = kz
            waves[c, ..., 3] = np.where(band, w, 0.0)
        # conjugate (InitialSpectrum.compute:135-143)
        my = (n - np.arange(n)) % n
        mirror = h0[:, my][:, :, my]
        h0[..., 2] = mirror[..., 0]
        h0[..., 3] = -mirror[..., 1]
        return h0, waves

    @staticmethod
    def evolve(h0, waves, t):
        hk = h0[..., 0] + 1j * h0[..., 1]
        hmk = h0[..., 2] + 1j * h0[..., 3]
        ph = waves[..., 3] * t
        e = np.exp(1j * ph)
        h = hk * e + hmk * np.conj(e)
        ih = 1j * h
        kx, ik, kz = waves[..., 0], waves[..., 1], waves[..., 2]
        Dx, Dz, Dy = ih * kx * ik, ih * kz * ik, h
        Dyx, Dyz = ih * kx, ih * kz
        aux = -h * ik
        Dxx, Dzz, Dxz = aux * kx * kx, aux * kz * kz, aux * kx * kz
        return [Dx + 1j * Dz, Dy + 1j * Dxz, Dyx + 1j * Dyz, Dxx + 1j * Dzz]

    @staticmethod
    def ifft2d(z):
        """N^2 * ifft2 with the (-1)^(x+y) permute; z complex [..., N, N] indexed [y][x]."""
        n = z.shape[-1]
        out = np.fft.ifft2(z, axes=(-2, -1)) * (n * n)
        yy, xx = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
        return out * (1 - 2 * ((xx + yy) % 2))

    @staticmethod
    def frame(h0, waves, t, turb_prev=None):
        P = [ref64.ifft2d(q) for q in ref64.evolve(h0, waves, t)]
        disp = np.stack([P[0].real, P[1].real, P[0].imag], -1)
        deriv = np.stack([P[2].real, P[2].imag, P[3].real, P[3].imag], -1)
        jac = (1 + P[3].real) * (1 + P[3].imag) - P[1].imag ** 2
        foam = (np.zeros_like(jac) if turb_prev is None else turb_prev) * float(FOAM_DECAY)
        foam = np.where(foam < jac, foam + jac, foam)
        return disp, deriv, foam


# ------------------------------------------------------------ world sampling
def _bil(u, v, m):
    """Bilinear tap coordinates on an m x m level (ocean.h ocean_sample_world), fp32."""
    f32 = np.float32
    fm = f32(m)
    inv = f32(1.0) / fm
    sx = u * fm - f32(0.5)
    sy = v * fm - f32(0.5)
    flx, fly = np.floor(sx), np.floor(sy)
    ix = (flx - fm * np.floor(flx * inv)).astype(np.int64)
    iy = (fly - fm * np.floor(fly * inv)).astype(np.int64)
    return ix, (ix + 1) & (m - 1), iy, (iy + 1) & (m - 1), sx - flx, sy - fly


def _lerp(a, b, f):
    return a + f[..., None] * (b - a)


def _tap(tex, u, v):
    """tex [m][m][4] float32, u/v float32[M] -> [M][4] (Repeat wrap, x then y)."""
    m = tex.shape[0]
    x0, x1, y0, y1, fx, fy = _bil(u, v, m)
    return _lerp(_lerp(tex[y0, x0], tex[y0, x1], fx), _lerp(tex[y1, x0], tex[y1, x1], fx), fy)


def _tri(levels, u, v, lod):
    """levels[0..log2 N] of one slice; lod float32[M] (None: level 0 only)."""
    if lod is None or len(levels) == 1:
        return _tap(levels[0], u, v)
    logn = len(levels) - 1
    out = _tap(levels[0], u, v)
    pos = lod > 0
    if pos.any():
        lc = np.minimum(lod[pos], np.float32(logn))
        l0 = np.floor(lc).astype(np.int64)
        l1 = np.minimum(l0 + 1, logn)
        f = lc - l0.astype(np.float32)
        a = np.empty((pos.sum(), 4), np.float32)
        b = np.empty_like(a)
        for lv in range(logn + 1):
            s0, s1 = l0 == lv, l1 == lv
            if s0.any():
                a[s0] = _tap(levels[lv], u[pos][s0], v[pos][s0])
            if s1.any():
                b[s1] = _tap(levels[lv], u[pos][s1], v[pos][s1])
        out[pos] = _lerp(a, b, f)
    return out


def sample_world(disp, deriv, turb, lengths, points, deriv_mips=None, turb_mips=None):
    """fp32 restatement of ocean_sample_world (Water.shader:314-348 with the library's stated
    filtering, include/ocean/ocean.h): disp/deriv/turb [C][N][N][4] of one tile (deriv/turb
    None for displacement-only), lengths [C], points [M][3] = (x, z, lod), optional mip
    chains as lists per cascade of levels 1..log2 N -> [M][3][4]."""
    f32 = np.float32
    pts = np.asarray(points, f32)
    x, z, lod = pts[:, 0], pts[:, 1], pts[:, 2]
    M = pts.shape[0]
    d_sum = np.zeros((M, 4), f32)
    g_sum = np.zeros((M, 4), f32)
    t_sum = np.zeros(M, f32)
    for c, L in enumerate(lengths):
        L = f32(L)
        u, v = x / L, z / L
        d_sum = d_sum + _tap(disp[c].astype(f32), u, v)
        if deriv is not None:
            dl = [deriv[c]] + (list(deriv_mips[c]) if deriv_mips is not None else [])
            tl = [turb[c]] + (list(turb_mips[c]) if turb_mips is not None else [])
            g_sum = g_sum + _tri(dl, u, v, lod if deriv_mips is not None else None)
            tb = _tri(tl, u, v, lod if turb_mips is not None else None)[:, 0]
            t_sum = t_sum + (f32(1.0) - np.minimum(np.maximum(tb, f32(0.0)), f32(1.0)))
    one = f32(1.0)
    sx = g_sum[:, 0] / (one + g_sum[:, 2])
    sz = g_sum[:, 1] / (one + g_sum[:, 3])
    inv = one / np.sqrt((sx * sx + one) + sz * sz)
    out = np.empty((M, 3, 4), f32)
    out[:, 0, :3] = d_sum[:, :3]
    out[:, 0, 3] = t_sum
    out[:, 1] = g_sum
    out[:, 2] = np.stack([-sx * inv, inv, -sz * inv, np.zeros_like(inv)], -1)
    return out


def scene_params(shallow: bool = False) -> dict:
    """WaterBody values from Assets/Scenes/Waves.unity:1305-1310 (depth 4 = script default, WaterBody.cs:14)."""
    return dict(wind_speed=8.0, wind_dir_x=1.0, wind_dir_y=-1.0, gravity=9.81, fetch=50000.0,
                depth=4.0 if shallow else 2560.0)


SCENE_CASCADES = [  # Waves.unity:1431-1435, 470-474, 1249-1253, 1572-1576
    dict(wavelength=1530.0, cutoff_low=1e-10, cutoff_high=1e12, swell=0.4, fade=0.1),
    dict(wavelength=1000.0, cutoff_low=1e-7, cutoff_high=1e7, swell=0.3, fade=0.2),
    dict(wavelength=201.0, cutoff_low=1e-5, cutoff_high=1e6, swell=0.1, fade=0.1),
    dict(wavelength=34.0, cutoff_low=0.001, cutoff_high=10.0, swell=0.4, fade=0.1),
]


def rel_err(a, b):
    """Norm-relative error max|a-b| / max|b| (DESIGN.md section 2 tolerance definition)."""
    a = np.asarray(a)
    b = np.asarray(b)
    den = np.abs(b).max()
    return float(np.abs(a - b).max() / (den if den > 0 else 1.0))


def pointwise_err(a, b, frac=1e-3):
    """SURVEY.md section 7's second tolerance clause: max |a-b| / |b| over the texels where
    |b| >= frac * max|b| (the near-zero texels excluded).  Returns (error, texels in the mask)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    mag = np.abs(b)
    m = mag >= frac * mag.max() if mag.max() > 0 else np.zeros(b.shape, bool)
    if not m.any():
        return 0.0, 0
    return float((np.abs(a[m] - b[m]) / mag[m]).max()), int(m.sum())
