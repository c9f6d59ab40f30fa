"""ocean_hip -- Python host mirror of the reference's WaterBody / IFFT interface
over liboceanhip.so (the MI355X C ABI declared in include/ocean/ocean.h).

The reference's host side is C# (Unity MonoBehaviours); no C# toolchain exists
in this image, so the host layer that the tests and the bench drive is this
ctypes binding, shaped like the reference:

    WaterBody  (Assets/Scripts/Water/WaterBody.cs)  -- fields, Awake(),
               CalculateWavesTexturesAtTime(t), Update(t), GetWaterHeight(pos)
    IFFT       (Assets/Scripts/Water/IFFT.cs)       -- InverseFastFourierTransform(plane)
    WaterCascade (Assets/Scripts/Water/WaterCascade.cs)

A compile-ready C# P/Invoke facade of the same ABI lives in ../csharp/ and in
INTEGRATION.md.  There is no CPU fallback: if the HIP library cannot be loaded
(or no GPU is present) every compute call raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

# torch is only plumbing here (device count, torch.distributed in bench.py), but
# its bundled HIP runtime must be the one this library binds to: import it first
# so that libamdhip64.so.7 resolves to the already-loaded copy (one runtime per
# process).
try:  # pragma: no cover - import side effect only
    import torch as _torch  # noqa: F401
except Exception:  # torch absent: the library then binds to /opt/rocm's runtime
    _torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OCEAN_HIP_LIB") or os.path.join(_HERE, "liboceanhip.so")

OK = 0
E_INVALID_ARG = -1
E_UNSUPPORTED = -2
E_STATE = -3
E_DEVICE = -4
E_OUT_OF_MEMORY = -5

F_DISPLACEMENT_ONLY = 0x1
F_NORMALS = 0x2
F_UNFUSED = 0x4
F_MIPS = 0x8

TEX_NOISE, TEX_H0, TEX_WAVES = 0, 1, 2
TEX_PLANE0, TEX_PLANE1, TEX_PLANE2, TEX_PLANE3 = 3, 4, 5, 6
TEX_DISP, TEX_DERIV, TEX_TURB, TEX_NORMAL = 7, 8, 9, 10
_TEX_CHANNELS = {TEX_NOISE: 2, TEX_H0: 4, TEX_WAVES: 4, TEX_PLANE0: 2, TEX_PLANE1: 2, TEX_PLANE2: 2,
                 TEX_PLANE3: 2, TEX_DISP: 4, TEX_DERIV: 4, TEX_TURB: 4, TEX_NORMAL: 4}

# symbols declared in include/ocean/ocean.h
EXPORTED_SYMBOLS = (
    "ocean_create", "ocean_destroy", "ocean_set_params", "ocean_set_noise", "ocean_generate_noise",
    "ocean_init_spectrum", "ocean_step", "ocean_evolve", "ocean_ifft2d", "ocean_fill", "ocean_read",
    "ocean_write", "ocean_get_device_ptr", "ocean_get_stream", "ocean_synchronize",
    "ocean_set_kernel_timing", "ocean_kernel_stats", "ocean_step_bytes", "ocean_read_mip", "ocean_get_mip_ptr",
    "ocean_generate_noise_device", "ocean_read_async", "ocean_readback_status", "ocean_readback_wait", "ocean_readback_release",
    "ocean_readback_copy_ms", "ocean_read_height_async", "ocean_set_readback_timing",
    "ocean_host_alloc", "ocean_host_free", "ocean_last_error", "ocean_abi_version", "ocean_set_column_band",
    "ocean_reset_foam", "ocean_sample_world", "ocean_sample_world_device", "ocean_kernel_name",
    "ocean_set_column_parity",
)


class OceanError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where} failed ({code}): {msg}")
        self.code = code


class ocean_params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in
                ("wind_speed", "wind_dir_x", "wind_dir_y", "gravity", "fetch", "depth")]


class ocean_cascade(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in ("wavelength", "cutoff_low", "cutoff_high", "swell", "fade")]


_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load liboceanhip.so (raises if it was not built -- there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OceanError(E_DEVICE, "load_library",
                         f"{path} not found: build it with `make -C ocean-simulation_amd` "
                         "(or __graft_entry__.build())")
    L = ctypes.CDLL(path)
    P = ctypes.c_void_p
    i, u32, u64, f, sz = ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_float, ctypes.c_size_t
    sig = {
        "ocean_create": ([i, i, i, i, u32, ctypes.POINTER(P)], i),
        "ocean_destroy": ([P], None),
        "ocean_set_params": ([P, ctypes.POINTER(ocean_params), ctypes.POINTER(ocean_cascade)], i),
        "ocean_set_noise": ([P, i, P], i),
        "ocean_generate_noise": ([P, u64], i),
        "ocean_init_spectrum": ([P], i),
        "ocean_reset_foam": ([P], i),
        "ocean_sample_world": ([P, i, P, i, P], i),
        "ocean_sample_world_device": ([P, i, P, i, P], i),
        "ocean_step": ([P, f], i),
        "ocean_evolve": ([P, f], i),
        "ocean_ifft2d": ([P, i], i),
        "ocean_fill": ([P], i),
        "ocean_read": ([P, i, i, i, P, sz], i),
        "ocean_write": ([P, i, i, i, P, sz], i),
        "ocean_get_device_ptr": ([P, i, ctypes.POINTER(P), ctypes.POINTER(sz)], i),
        "ocean_get_stream": ([P, ctypes.POINTER(P)], i),
        "ocean_synchronize": ([P], i),
        "ocean_set_kernel_timing": ([P, i], i),
        "ocean_kernel_stats": ([P, i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong)], i),
        "ocean_kernel_name": ([P, i, ctypes.c_char_p, sz], i),
        "ocean_step_bytes": ([P, ctypes.POINTER(u64), ctypes.POINTER(u64)], i),
        "ocean_read_mip": ([P, i, i, i, i, P, sz], i),
        "ocean_generate_noise_device": ([P, u64], i),
        "ocean_get_mip_ptr": ([P, i, i, ctypes.POINTER(P), ctypes.POINTER(sz)], i),
        "ocean_read_async": ([P, i, i, i, P, sz, ctypes.POINTER(P)], i),
        "ocean_readback_status": ([P], i),
        "ocean_readback_wait": ([P], i),
        "ocean_readback_release": ([P], None),
        "ocean_readback_copy_ms": ([P, ctypes.POINTER(f)], i),
        "ocean_read_height_async": ([P, i, i, P, sz, ctypes.POINTER(P)], i),
        "ocean_set_readback_timing": ([P, i], i),
        "ocean_host_alloc": ([sz, ctypes.POINTER(P)], i),
        "ocean_host_free": ([P], None),
        "ocean_last_error": ([], ctypes.c_char_p),
        "ocean_abi_version": ([], i),
        "ocean_set_column_band": ([P, i, i], i),
        "ocean_set_column_parity": ([P, i], i),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def _check(rc: int, where: str) -> None:
    if rc != OK:
        msg = load_library().ocean_last_error().decode(errors="replace")
        raise OceanError(rc, where, msg)


class OceanContext:
    """Thin owner of one ocean_ctx (one device, T tiles x C cascades at N x N)."""

    def __init__(self, n: int, n_cascades: int, n_tiles: int = 1, flags: int = 0, device: int = 0):
        self.lib = load_library()
        self.n, self.C, self.T, self.flags, self.device = n, n_cascades, n_tiles, flags, device
        self.planes = 2 if flags & F_DISPLACEMENT_ONLY else 4
        h = ctypes.c_void_p()
        _check(self.lib.ocean_create(device, n, n_cascades, n_tiles, flags, ctypes.byref(h)), "ocean_create")
        self._h = h

    # -- lifetime -----------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.ocean_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- configuration --------------------------------------------------------
    def set_params(self, params: dict, cascades: Sequence[dict]) -> None:
        if len(cascades) != self.C:
            raise ValueError(f"expected {self.C} cascades, got {len(cascades)}")
        p = ocean_params(params["wind_speed"], params["wind_dir_x"], params["wind_dir_y"], params["gravity"],
                         params["fetch"], params["depth"])
        cs = (ocean_cascade * self.C)(*[ocean_cascade(c["wavelength"], c["cutoff_low"], c["cutoff_high"],
                                                      c["swell"], c["fade"]) for c in cascades])
        _check(self.lib.ocean_set_params(self._h, ctypes.byref(p), cs), "ocean_set_params")

    def set_noise(self, tile: int, rg: np.ndarray) -> None:
        a = np.ascontiguousarray(rg, np.float32)
        if a.shape != (self.n, self.n, 2):
            raise ValueError(f"noise must be float32[{self.n}][{self.n}][2], got {a.shape}")
        _check(self.lib.ocean_set_noise(self._h, tile, a.ctypes.data), "ocean_set_noise")

    def generate_noise(self, seed: int) -> None:
        _check(self.lib.ocean_generate_noise(self._h, ctypes.c_uint64(seed)), "ocean_generate_noise")

    # -- compute --------------------------------------------------------------
    def generate_noise_device(self, seed: int) -> None:
        """Counter-based noise generated on the GPU for every tile (ocean.h)."""
        _check(self.lib.ocean_generate_noise_device(self._h, seed), "ocean_generate_noise_device")

    def init_spectrum(self) -> None:
        _check(self.lib.ocean_init_spectrum(self._h), "ocean_init_spectrum")

    def reset_foam(self) -> None:
        _check(self.lib.ocean_reset_foam(self._h), "ocean_reset_foam")

    def step(self, t: float) -> None:
        _check(self.lib.ocean_step(self._h, ctypes.c_float(t)), "ocean_step")

    def evolve(self, t: float) -> None:
        _check(self.lib.ocean_evolve(self._h, ctypes.c_float(t)), "ocean_evolve")

    def ifft2d(self, plane_mask: int) -> None:
        _check(self.lib.ocean_ifft2d(self._h, plane_mask), "ocean_ifft2d")

    def fill(self) -> None:
        _check(self.lib.ocean_fill(self._h), "ocean_fill")

    def synchronize(self) -> None:
        _check(self.lib.ocean_synchronize(self._h), "ocean_synchronize")

    # -- textures -------------------------------------------------------------
    def read(self, tex: int, tile: int = 0, cascade: int = 0) -> np.ndarray:
        ch = _TEX_CHANNELS[tex]
        out = np.empty((self.n, self.n, ch), np.float32)
        _check(self.lib.ocean_read(self._h, tex, tile, cascade, out.ctypes.data, out.nbytes), "ocean_read")
        return out

    def read_all(self, tex: int, tile: int = 0) -> np.ndarray:
        return np.stack([self.read(tex, tile, c) for c in range(self.C)])

    def write(self, tex: int, data: np.ndarray, tile: int = 0, cascade: int = 0) -> None:
        a = np.ascontiguousarray(data, np.float32)
        _check(self.lib.ocean_write(self._h, tex, tile, cascade, a.ctypes.data, a.nbytes), "ocean_write")

    def read_mip(self, tex: int, level: int, tile: int = 0, cascade: int = 0) -> np.ndarray:
        """Level `level` of DERIV / TURB's mip chain (OCEAN_F_MIPS); level 0 = read()."""
        m = self.n >> level
        out = np.empty((m, m, 4), np.float32)
        _check(self.lib.ocean_read_mip(self._h, tex, tile, cascade, level, out.ctypes.data, out.nbytes),
               "ocean_read_mip")
        return out

    def mip_ptr(self, tex: int, level: int):
        """(device pointer of level `level` of slice 0, bytes between slices' chains)."""
        p, st = ctypes.c_void_p(), ctypes.c_size_t()
        _check(self.lib.ocean_get_mip_ptr(self._h, tex, level, ctypes.byref(p), ctypes.byref(st)), "ocean_get_mip_ptr")
        return p.value, st.value

    def sample_world(self, points: np.ndarray, tile: int = 0) -> np.ndarray:
        """Cascade-summed world sampling (Water.shader:314-348; ocean.h ocean_sample_world):
        points float[M][3] = (world x, world z, lod) -> float32[M][3][4]: (Dx, Dy, Dz,
        turbulence), (Dyx, Dyz, Dxx, Dzz), (normal x, y, z, 0)."""
        p = np.ascontiguousarray(points, np.float32)
        if p.ndim != 2 or p.shape[1] != 3:
            raise ValueError(f"points must be float32[M][3], got {p.shape}")
        out = np.empty((p.shape[0], 3, 4), np.float32)
        _check(self.lib.ocean_sample_world(self._h, tile, p.ctypes.data, p.shape[0], out.ctypes.data),
               "ocean_sample_world")
        return out

    def read_async(self, tex: int, tile: int = 0, cascade: int = 0, buf: "PinnedBuffer" = None) -> "Readback":
        """AsyncGPUReadback.Request (WaterBody.cs:288-296): copy one slice into pinned
        host memory once the queued steps finish; poll .done() / .wait(), then .data.
        `buf`: a caller-owned pinned slot to land in (else the request allocates its own)."""
        return Readback(self, tex, tile, cascade, buf)

    def read_height_async(self, tile: int = 0, cascade: int = 0, buf: "PinnedBuffer" = None) -> "Readback":
        """The height-only readback (ocean_read_height_async): DISP.y of one slice as float32[N][N], a
        quarter of read_async(TEX_DISP)'s bytes -- all GetWaterHeight reads (WaterBody.cs:195-209)."""
        return Readback(self, TEX_DISP, tile, cascade, buf, height=True)

    def set_readback_timing(self, enable: bool) -> None:
        """Time each new readback's device-to-host copy (Readback.copy_ms); off after create."""
        _check(self.lib.ocean_set_readback_timing(self._h, 1 if enable else 0), "ocean_set_readback_timing")

    def device_ptr(self, tex: int):
        p, b = ctypes.c_void_p(), ctypes.c_size_t()
        _check(self.lib.ocean_get_device_ptr(self._h, tex, ctypes.byref(p), ctypes.byref(b)), "ocean_get_device_ptr")
        return p.value, b.value

    def stream(self) -> int:
        s = ctypes.c_void_p()
        _check(self.lib.ocean_get_stream(self._h, ctypes.byref(s)), "ocean_get_stream")
        return s.value or 0

    def set_column_band(self, x_begin: int, x_count: int) -> None:
        """Restrict the fused step's stores, column transforms and fill to columns
        [x_begin, x_begin + x_count) (one GPU's share of a unit split over several)."""
        _check(self.lib.ocean_set_column_band(self._h, x_begin, x_count), "ocean_set_column_band")

    def set_column_parity(self, parity: int) -> None:
        """Compute only the columns x = 2m + parity (stored compact at texture column m < N/2):
        one of two GPUs sharing a unit with no duplicated row transform (ocean.h); -1 = off."""
        _check(self.lib.ocean_set_column_parity(self._h, parity), "ocean_set_column_parity")

    # -- timing ---------------------------------------------------------------
    def set_kernel_timing(self, enable: bool) -> None:
        _check(self.lib.ocean_set_kernel_timing(self._h, 1 if enable else 0), "ocean_set_kernel_timing")

    def kernel_stats(self, kind: int):
        ms, cnt = ctypes.c_double(), ctypes.c_longlong()
        _check(self.lib.ocean_kernel_stats(self._h, kind, ctypes.byref(ms), ctypes.byref(cnt)), "ocean_kernel_stats")
        return ms.value, cnt.value

    def kernel_name(self, kind: int) -> Optional[str]:
        """Demangled symbol of the kernel this context launched last in `kind` (0 pass A / rows,
        1 pass B / columns, 2 other), as rocprofv3 names it; None before any such launch."""
        buf = ctypes.create_string_buffer(1024)
        rc = self.lib.ocean_kernel_name(self._h, kind, buf, len(buf))
        if rc == E_STATE:
            return None
        _check(rc, "ocean_kernel_name")
        return buf.value.decode()

    def step_bytes(self):
        """(pass A, pass B) algorithmic HBM bytes of one step in this context's schedule."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self.lib.ocean_step_bytes(self._h, ctypes.byref(a), ctypes.byref(b)), "ocean_step_bytes")
        return a.value, b.value


class PinnedBuffer:
    """Pinned host memory from ocean_host_alloc, freed by release() (hipHostFree synchronizes the
    device, so a host that reads back every frame allocates its slots once and reuses them)."""

    def __init__(self, nbytes: int):
        self.lib = load_library()
        self.nbytes = nbytes
        self.ptr = ctypes.c_void_p()
        _check(self.lib.ocean_host_alloc(nbytes, ctypes.byref(self.ptr)), "ocean_host_alloc")

    def release(self) -> None:
        if self.ptr:
            self.lib.ocean_host_free(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.release()
        except Exception:
            pass


class Readback:
    """One ocean_read_async (or, `height`, ocean_read_height_async) request into pinned host memory:
    a caller's PinnedBuffer slot, or one of its own (freed by release())."""

    def __init__(self, ctx: "OceanContext", tex: int, tile: int, cascade: int, buf: Optional[PinnedBuffer] = None,
                 height: bool = False):
        self.lib = ctx.lib
        ch = 1 if height else _TEX_CHANNELS[tex]
        self.shape = (ctx.n, ctx.n) if height else (ctx.n, ctx.n, ch)
        self.nbytes = ctx.n * ctx.n * ch * 4
        self._h = ctypes.c_void_p()
        self.slot = buf
        self._own = buf is None
        if buf is None:
            buf = PinnedBuffer(self.nbytes)
        elif buf.nbytes < self.nbytes:
            raise ValueError(f"pinned slot of {buf.nbytes} B < slice {self.nbytes} B")
        self._pinned = buf
        self._buf = buf.ptr
        if height:
            rc = self.lib.ocean_read_height_async(ctx._h, tile, cascade, self._buf, self.nbytes, ctypes.byref(self._h))
        else:
            rc = self.lib.ocean_read_async(ctx._h, tex, tile, cascade, self._buf, self.nbytes, ctypes.byref(self._h))
        if rc != OK:
            if self._own:
                buf.release()
            self._pinned = None
            self._buf = ctypes.c_void_p()
            _check(rc, "ocean_read_height_async" if height else "ocean_read_async")

    def done(self) -> bool:
        rc = self.lib.ocean_readback_status(self._h)
        if rc < 0:
            _check(rc, "ocean_readback_status")
        return rc == 1

    def wait(self) -> None:
        _check(self.lib.ocean_readback_wait(self._h), "ocean_readback_wait")

    def copy_ms(self) -> float:
        """The completed request's device-to-host copy duration (ocean_readback_copy_ms; the request must
        have been made with readback timing on: OceanContext.set_readback_timing)."""
        ms = ctypes.c_float()
        _check(self.lib.ocean_readback_copy_ms(self._h, ctypes.byref(ms)), "ocean_readback_copy_ms")
        return ms.value

    @property
    def data(self) -> np.ndarray:
        """A copy of the completed readback (waits if still pending)."""
        return self.view().copy()

    def view(self) -> np.ndarray:
        """The completed readback in place, read-only, without a copy (waits if still pending).  Valid
        while the pinned slot is neither released nor handed to another request."""
        self.wait()
        raw = (ctypes.c_float * (self.nbytes // 4)).from_address(self._buf.value)
        v = np.frombuffer(raw, np.float32).reshape(self.shape)
        v.flags.writeable = False
        return v

    def release(self) -> None:
        if self._h:
            self.lib.ocean_readback_release(self._h)
            self._h = ctypes.c_void_p()
        if self._pinned is not None and self._own:
            self._pinned.release()
        self._pinned = None
        self._buf = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.release()
        except Exception:
            pass


# ---------------------------------------------------------------------------
# Reference-shaped facade
# ---------------------------------------------------------------------------
@dataclass
class WaterCascade:
    """WaterCascade.cs:10-24 (defaults from the script)."""
    wavelength: float = 10.0
    cutoffHigh: float = 5.0
    cutoffLow: float = 0.0001
    swell: float = 0.4
    fade: float = 0.1

    def as_dict(self) -> dict:
        return dict(wavelength=self.wavelength, cutoff_low=self.cutoffLow, cutoff_high=self.cutoffHigh,
                    swell=self.swell, fade=self.fade)


@dataclass
class WaterBody:
    """WaterBody.cs public surface over the HIP library.

    Fields and defaults follow WaterBody.cs:10-33.  Awake() allocates and runs
    the initial spectrum (WaterBody.cs:211-256); CalculateWavesTexturesAtTime(t)
    is the per-frame path (WaterBody.cs:180-193, mip chains of DERIV and TURB
    included when `mips`); Update(t) additionally requests displacement slice 0
    asynchronously and, once a request completes, refreshes buoyancyData for
    GetWaterHeight (AsyncGPUReadback, WaterBody.cs:284-297, 195-209).
    `tiles` > 1 batches independent oceans (tile k uses seed + k).
    `readback`: "height" (default) requests only the .g channel GetWaterHeight reads
    (ocean_read_height_async, 4 B per texel: the reference's buoyancyData is private,
    WaterBody.cs:58, and that is its only reader); "rgba" requests the whole Color slice
    (16 B per texel) as the reference does.  GetWaterHeight returns the same bits in both.
    """
    windSpeed: float = 1.0
    windDirection: tuple = (1.0, 1.0)
    gravity: float = 9.81
    fetch: float = 1.0
    depth: float = 4.0
    texturesSize: int = 256
    cascades: List[WaterCascade] = field(default_factory=lambda: [WaterCascade()])
    seed: int = 20251121
    tiles: int = 1
    displacementOnly: bool = False
    normals: bool = False
    mips: bool = True  # WaterBody.cs:228-229 creates DERIV / TURB with mip chains
    device: int = 0
    noise: Optional[np.ndarray] = None  # explicit noise texture (tile 0), float32[N][N][2]
    readback: str = "height"  # "height" (DISP.y only) or "rgba" (the whole displacement slice)

    def __post_init__(self):
        self.ctx: Optional[OceanContext] = None
        self._buoy: Optional[np.ndarray] = None  # the last landed slice: a view of the held pinned slot
        self._readbacks: List[Readback] = []
        self._ring: List[PinnedBuffer] = []  # pinned readback slots, allocated in Awake
        self._idle: List[PinnedBuffer] = []
        self._held: Optional[PinnedBuffer] = None  # the pinned slot the last landed slice stays in
        self._buoy_copy: Optional[np.ndarray] = None  # buoyancyData's copy of the landed slice (first access)
        self.readback_copy_ms: Optional[List[float]] = None  # set to [] to log each landed copy's time
        self._timed = False  # the context's readback timing (on while readback_copy_ms is a list)

    def params(self) -> dict:
        return dict(wind_speed=self.windSpeed, wind_dir_x=self.windDirection[0], wind_dir_y=self.windDirection[1],
                    gravity=self.gravity, fetch=self.fetch, depth=self.depth)

    def Awake(self) -> "WaterBody":
        flags = (F_DISPLACEMENT_ONLY if self.displacementOnly else 0) | (F_NORMALS if self.normals else 0)
        if self.mips and not self.displacementOnly:
            flags |= F_MIPS
        self.ctx = OceanContext(self.texturesSize, len(self.cascades), self.tiles, flags, self.device)
        self.ctx.set_params(self.params(), [c.as_dict() for c in self.cascades])
        if self.noise is not None:
            self.ctx.set_noise(0, self.noise)
            for t in range(1, self.tiles):
                self.ctx.set_noise(t, self.noise)
        else:
            self.ctx.generate_noise(self.seed)
        self.ctx.init_spectrum()
        if self.readback not in ("height", "rgba"):
            raise ValueError(f"readback must be 'height' or 'rgba', got {self.readback!r}")
        self._timed = False
        slice_bytes = self.texturesSize * self.texturesSize * (4 if self.readback == "height" else 16)
        # one slot more than the requests in flight: the one the last landed slice stays in
        self._ring = [PinnedBuffer(slice_bytes) for _ in range(self._in_flight() + 1)]
        self._idle = list(self._ring)
        self._held = None
        return self

    def OnValidate(self) -> None:
        """Parameter change -> spectrum re-init (the commented OnValidate, WaterBody.cs:324-337);
        the foam accumulator carries over, as there."""
        self.ctx.set_params(self.params(), [c.as_dict() for c in self.cascades])
        self.ctx.init_spectrum()

    def CalculateWavesTexturesAtTime(self, time: float) -> None:
        self.ctx.step(time)

    # Bound on queued requests (the reference's queue is engine-managed); the ring holds one pinned slot
    # more, the one the last landed slice stays in.  Measured at cfg3 (tools/readback_probe.py): 2-4 in
    # flight keep the 16 MiB copies back to back beside the frames, 0.33 ms per frame; 8 in flight run
    # 0.82 ms per frame, each copy stretched to 2.5x its time alone.
    MAX_READBACKS_IN_FLIGHT = 4

    def _in_flight(self) -> int:
        """The bound in force: at least one request (water_body.h clamps the same way)."""
        return max(int(self.MAX_READBACKS_IN_FLIGHT), 1)

    def Update(self, time: float) -> None:
        """WaterBody.Update (WaterBody.cs:284-297): step, then issue a new AsyncGPUReadback
        request of displacement slice 0 EVERY frame (:288); requests complete in order and
        each completed one refreshes buoyancyData, as the reference's callback does (:292-295)."""
        self.CalculateWavesTexturesAtTime(time)
        self._poll_readbacks()
        # at most MAX_READBACKS_IN_FLIGHT requests queued (the ring's extra slot holds the landed slice):
        # when full, wait for the oldest
        while self._readbacks and (len(self._readbacks) >= self._in_flight() or not self._idle):
            self._complete(self._readbacks.pop(0))
        if (self.readback_copy_ms is not None) != self._timed:  # copy times logged: timed requests
            self._timed = self.readback_copy_ms is not None
            self.ctx.set_readback_timing(self._timed)
        slot = self._idle.pop()
        try:
            if self.readback == "height":
                rb = self.ctx.read_height_async(0, 0, slot)
            else:
                rb = self.ctx.read_async(TEX_DISP, 0, 0, slot)
            rb.timed = self._timed
            self._readbacks.append(rb)
        except Exception:
            self._idle.append(slot)
            raise

    def _complete(self, rb: "Readback") -> None:
        # The reference copies every completed request out (request.GetData<Color>().ToArray(),
        # WaterBody.cs:295): Unity's NativeArray lives only inside the callback.  A pinned ring slot
        # outlives its request, so the landed slice stays in place instead: the slot leaves the
        # ring until the next completed readback replaces it, GetWaterHeight reads it there, and
        # buoyancyData copies it out only when a caller asks (16 MiB of host copy saved per frame
        # at 1024^2).
        view = rb.view()
        if self.readback_copy_ms is not None and rb.timed:
            self.readback_copy_ms.append(rb.copy_ms())
        slot = rb.slot
        rb.release()
        if self._held is not None:
            self._idle.append(self._held)
        self._held = slot
        self._buoy = view
        self._buoy_copy = None

    @property
    def buoyancyData(self) -> Optional[np.ndarray]:
        """The last landed displacement slice 0 (WaterBody.cs:295's array), read-only: [y][x] heights
        (.g) with readback "height", [y][x][rgba] with "rgba".
        The slice is copied out of its pinned slot once, on the first access after it lands, and the
        same array is returned until the next readback lands: per-sample indexing costs no copy, as
        reading the reference's field does not."""
        if self._buoy is None:
            return None
        if self._buoy_copy is None:
            self._buoy_copy = np.array(self._buoy)
            self._buoy_copy.flags.writeable = False
        return self._buoy_copy

    def _poll_readbacks(self) -> None:
        while self._readbacks and self._readbacks[0].done():
            self._complete(self._readbacks.pop(0))

    def WaitForReadback(self) -> None:
        """Block until every pending readback has landed (the last one in buoyancyData)."""
        while self._readbacks:
            self._complete(self._readbacks.pop(0))

    def GetWaterHeight(self, worldPosition) -> float:
        """WaterBody.cs:195-209, including its quirk of mapping world x,z over
        [-texturesSize/2, texturesSize/2] instead of the cascade length."""
        if self._buoy is None:
            return 0.0
        n = self.texturesSize

        def inv_lerp(a, b, v):
            return 0.0 if a == b else min(max((v - a) / (b - a), 0.0), 1.0)
        u = inv_lerp(-(n // 2), n // 2, float(worldPosition[0]))
        v = inv_lerp(-(n // 2), n // 2, float(worldPosition[2]))
        x = min(max(int(u * n), 0), n - 1)
        y = min(max(int(v * n), 0), n - 1)
        return float(self._buoy[y, x] if self.readback == "height" else self._buoy[y, x, 1])

    def SampleWorld(self, points, tile: int = 0) -> np.ndarray:
        """What Water.shader reads at world positions (x, z, lod): summed displacement,
        derivatives, turbulence and the normal (Water.shader:314-348)."""
        return self.ctx.sample_world(np.asarray(points, np.float32).reshape(-1, 3), tile)

    # texture-out contract (material properties, WaterBody.cs:277-281)
    def DisplacementsTextures(self, tile: int = 0) -> np.ndarray:
        return self.ctx.read_all(TEX_DISP, tile)

    def DerivativesTextures(self, tile: int = 0) -> np.ndarray:
        return self.ctx.read_all(TEX_DERIV, tile)

    def TurbulenceTextures(self, tile: int = 0) -> np.ndarray:
        return self.ctx.read_all(TEX_TURB, tile)

    def OnDisable(self) -> None:
        for rb in self._readbacks:
            rb.release()
        self._readbacks = []
        if self._buoy is not None:  # the last landed slice outlives the pinned ring
            self._buoy = self.buoyancyData
        for b in self._ring:
            b.release()
        self._ring, self._idle, self._held = [], [], None
        if self.ctx is not None:
            self.ctx.close()
            self.ctx = None


class IFFT:
    """IFFT.cs operator: InverseFastFourierTransform on a plane texture array of a context."""

    def __init__(self, ctx: OceanContext):
        self.ctx = ctx

    def InverseFastFourierTransform(self, plane: int) -> None:
        """plane in 0..3 (DxDz, DyDxz, DyxDyz, DxxDzz): in-place, all tiles and cascades."""
        self.ctx.ifft2d(1 << plane)


def scene_water_body(n: int = 512, n_cascades: int = 3, **kw) -> WaterBody:
    """The reference scene (Assets/Scenes/Waves.unity:1305-1322, cascades :1431-1435, :470-474,
    :1249-1253, 4th unreferenced cascade :1572-1576)."""
    cs = [WaterCascade(1530, 1e12, 1e-10, 0.4, 0.1), WaterCascade(1000, 1e7, 1e-7, 0.3, 0.2),
          WaterCascade(201, 1e6, 1e-5, 0.1, 0.1), WaterCascade(34, 10, 0.001, 0.4, 0.1)][:n_cascades]
    return WaterBody(windSpeed=8.0, windDirection=(1.0, -1.0), gravity=9.81, fetch=50000.0, depth=2560.0,
                     texturesSize=n, cascades=cs, **kw)
