/*
 * ocean.h -- C ABI of liboceanhip.so, the MI355X (gfx950) implementation of the
 * reference's per-frame Tessendorf ocean path (Mozobo/Ocean-Simulation).
 *
 * The reference boundary is Unity's ComputeShader binding API driven from C#:
 * WaterBody.cs binds textures/buffers by string name and Dispatch()es the
 * InitialSpectrum / TimeDependentSpectrum / IFFT / ResultTexturesFiller kernels,
 * and the output stays in Tex2DArray RenderTextures read by Water.shader and by
 * AsyncGPUReadback (WaterBody.cs:180-193, :288-296).  Each entry point below
 * names the reference interface it replaces.  A C# P/Invoke binding of every
 * symbol is given in INTEGRATION.md.
 *
 * Conventions
 *   - cdecl, every struct blittable (LayoutKind.Sequential in C#).
 *   - Every int-returning call returns OCEAN_OK (0) or a negative OCEAN_E_*;
 *     no C++ exception crosses the ABI.  ocean_last_error() gives a
 *     thread-local message for the last failure on the calling thread.
 *   - The context owns all device memory; the caller owns host buffers, which
 *     are only read/written during the call.
 *   - GPU work is enqueued on the context's own HIP stream (one per ctx); only
 *     ocean_read / ocean_write / ocean_synchronize / ocean_set_noise /
 *     ocean_generate_noise block the calling thread.
 *   - A context is not thread-safe: drive it from one thread (like Unity's
 *     main thread).  Multi-GPU = one context per device.
 *   - The calling thread's current HIP device is never changed: a call makes
 *     its context's device current for the span of the call and restores the
 *     caller's device before it returns (ocean_create / ocean_destroy /
 *     ocean_readback_release included).  One thread may drive contexts on
 *     several devices, beside torch or any other HIP user, in any order.
 *
 * Memory layout in HBM (all fp32, texture index = [unit][y][x], unit = tile*C + cascade,
 * matching Unity's Tex2DArray [slice][y][x] with id.x = x):
 *   NOISE  float2 [T][N][N]       H0    float4 [T*C][N][N]   WAVES float4 [T*C][N][N]
 *   PLANEp float2 [T*C][N][N]     p = 0 DxDz, 1 DyDxz, 2 DyxDyz, 3 DxxDzz
 *   DISP   float4 [T*C][N][N]     DERIV float4 [T*C][N][N]  TURB  float4 [T*C][N][N]
 *   NORMAL float4 [T*C][N][N]     (derived output, OCEAN_F_NORMALS only)
 */
#ifndef OCEAN_OCEAN_H
#define OCEAN_OCEAN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Version history (a host checks ocean_abi_version() at load time):
 *   1  round-1 entry points.
 *   2  semantics changed: ocean_set_params only stages values until ocean_init_spectrum;
 *      ocean_init_spectrum no longer zeroes the foam (ocean_reset_foam does); ocean_write
 *      of OCEAN_TEX_WAVES is E_UNSUPPORTED without OCEAN_F_UNFUSED; ocean_sample_world*
 *      return E_STATE before ocean_init_spectrum and the device entry checks alignment.
 *      New: ocean_reset_foam, ocean_set_column_band, ocean_sample_world(_device),
 *      ocean_read_async family, ocean_host_alloc/free, ocean_generate_noise_device,
 *      ocean_kernel_name, ocean_set_column_parity.
 *   3  semantics changed: no call moves the calling thread's current HIP device any more
 *      (Conventions).  New: ocean_readback_copy_ms.
 *   4  semantics changed: ocean_readback_copy_ms needs a request made with readback timing on
 *      (ocean_set_readback_timing; off by default, so a host that never asks for copy times
 *      records no timing events).  New: ocean_read_height_async, ocean_set_readback_timing. */
#define OCEAN_ABI_VERSION 4

/* status codes */
#define OCEAN_OK 0
#define OCEAN_E_INVALID_ARG (-1)   /* bad pointer, size, index or enum */
#define OCEAN_E_UNSUPPORTED (-2)   /* N not a power of two in [16, 4096], C not in [1, 5], ... */
#define OCEAN_E_STATE (-3)         /* call order violated (e.g. step before init_spectrum) */
#define OCEAN_E_DEVICE (-4)        /* HIP runtime / kernel launch failure */
#define OCEAN_E_OUT_OF_MEMORY (-5) /* hipMalloc failed */

/* ocean_create flags */
#define OCEAN_F_DISPLACEMENT_ONLY 0x1u /* 2 planes (DxDz, DyDxz) -> DISP only (BASELINE cfg2) */
#define OCEAN_F_NORMALS 0x2u           /* also write the per-cascade NORMAL texture (Water.shader:346-348) */
#define OCEAN_F_UNFUSED 0x4u           /* ocean_step runs the reference-shaped schedule:
                                          evolve -> 4 x ifft2d -> fill (WaterBody.cs:180-190) */
#define OCEAN_F_MIPS 0x8u              /* allocate mip chains for DERIV and TURB and regenerate them
                                          in every ocean_step (WaterBody.cs:191-192, :228-229) */

/* texture ids for ocean_read / ocean_write / ocean_get_device_ptr */
enum ocean_texture {
    OCEAN_TEX_NOISE = 0,  /* _RandomNoiseTexture           WaterBody.cs:86-100 (per tile, cascade ignored) */
    OCEAN_TEX_H0 = 1,     /* _InitialSpectrumTextures      InitialSpectrum.compute:14 */
    OCEAN_TEX_WAVES = 2,  /* _WavesDataTextures            InitialSpectrum.compute:15 */
    OCEAN_TEX_PLANE0 = 3, /* _DxDzTextures                 TimeDependentSpectrum.compute:6 */
    OCEAN_TEX_PLANE1 = 4, /* _DyDxzTextures */
    OCEAN_TEX_PLANE2 = 5, /* _DyxDyzTextures */
    OCEAN_TEX_PLANE3 = 6, /* _DxxDzzTextures */
    OCEAN_TEX_DISP = 7,   /* _DisplacementsTextures        ResultTexturesFiller.compute:7 */
    OCEAN_TEX_DERIV = 8,  /* _DerivativesTextures          ResultTexturesFiller.compute:8 */
    OCEAN_TEX_TURB = 9,   /* _TurbulenceTextures (foam state) ResultTexturesFiller.compute:9 */
    OCEAN_TEX_NORMAL = 10 /* derived: normalize(-Dyx/(1+Dxx), 1, -Dyz/(1+Dzz)), w = 0 */
};

typedef struct ocean_ctx ocean_ctx;

/* WaterBody public ocean parameters, WaterBody.cs:10-14. */
typedef struct ocean_params {
    float wind_speed;
    float wind_dir_x;
    float wind_dir_y;
    float gravity;
    float fetch;
    float depth;
} ocean_params;

/* WaterCascade component, WaterCascade.cs:10-24 (flattened as WaterBody.cs:231-242). */
typedef struct ocean_cascade {
    float wavelength; /* patch length L */
    float cutoff_low;
    float cutoff_high;
    float swell;
    float fade;
} ocean_cascade;

/* Replaces WaterBody.Awake resource creation (WaterBody.cs:211-251) and
 * new IFFT(...) (IFFT.cs:24-62): allocates every texture for `n_tiles`
 * independent oceans of `n_cascades` cascades at N = `n` on HIP device
 * `device`, and builds the twiddle table.  16 <= n <= 4096, power of two;
 * 1 <= n_cascades <= 5 (Water.shader:139); n_tiles >= 1. */
int ocean_create(int device, int n, int n_cascades, int n_tiles, uint32_t flags, ocean_ctx **out);

/* Replaces OnDisable (WaterBody.cs:300-309) + RT release.  NULL is a no-op. */
void ocean_destroy(ocean_ctx *ctx);

/* Replaces the SetFloat/SetBuffer parameter bindings of
 * InitializeInitialSpectrumComputeShader (WaterBody.cs:130-148).
 * `cascades` has n_cascades entries.  The values are only staged: they take effect
 * at the next ocean_init_spectrum, and frames stepped before it keep running with
 * the previous spectrum's constants (fused and unfused alike). */
int ocean_set_params(ocean_ctx *ctx, const ocean_params *params, const ocean_cascade *cascades);

/* Replaces GenerateRandomNoiseTexture + Texture2D.Apply (WaterBody.cs:86-100, :97):
 * uploads tile `tile`'s noise, float2[N][N] laid out [y][x] (g1, g2). Blocking. */
int ocean_set_noise(ocean_ctx *ctx, int tile, const float *rg);

/* This library's documented, seeded noise (the reference's UnityEngine.Random is
 * unseeded and closed): tile t uses seed + t; Marsaglia polar over xorshift128
 * seeded by splitmix64, texels generated x-outer / y-inner, g1 then g2
 * (WaterBody.cs:71-100).  Generated on the host, uploaded.  Blocking. */
int ocean_generate_noise(ocean_ctx *ctx, uint64_t seed);

/* On-device noise for large tile batches (replaces the CPU
 * loop of WaterBody.cs:86-100): a counter-based generator, one independent stream
 * per texel -- a different sequence from ocean_generate_noise.  Texel (x, y) of
 * tile t: key = mix(seed + t + G) ^ ((y*N + x) * 0xD1B54A32D192ED03), uniform k
 * (k = 1, 2, ...) = (mix(key + k*G) >> 40) * 2^-24 with G = 0x9E3779B97F4A7C15 and
 * mix the splitmix64 finaliser; g1 then g2 each from the Marsaglia polar loop
 * (WaterBody.cs:71-81).  Blocking. */
int ocean_generate_noise_device(ocean_ctx *ctx, uint64_t seed);

/* Replaces CalculateInitialSpectrumTextures (WaterBody.cs:171-178):
 * InitialSpectrum.compute:99-129 then :135-143 for every tile and cascade, with
 * the parameters staged by ocean_set_params.  The foam state (TURB) is left as it
 * is, as in the reference's re-init on a parameter change (the commented
 * OnValidate, WaterBody.cs:324-337); it is zero after ocean_create.  Blocks until
 * the staged constants are on the device, then runs async on the ctx stream. */
int ocean_init_spectrum(ocean_ctx *ctx);

/* Zeroes the foam accumulator (TURB, its mip chain and the internal foam state)
 * of every tile and cascade, stream-ordered.  No reference counterpart: there the
 * RenderTexture starts zeroed once (WaterBody.cs:229) and is never cleared. */
int ocean_reset_foam(ocean_ctx *ctx);

/* Replaces CalculateWavesTexturesAtTime(time) (WaterBody.cs:180-193, minus
 * GenerateMips): evolve -> 2D IFFT of every plane -> fill/foam for all tiles
 * and cascades.  Async on the ctx stream.  Fused 2-kernel schedule by default;
 * OCEAN_F_UNFUSED selects the reference-shaped one (same results to rounding). */
int ocean_step(ocean_ctx *ctx, float time);

/* Column band for splitting one (tile, cascade) unit over several GPUs (SURVEY.md 8e,
 * "units < GPUs", cfg5 = 4 cascades on 8 GPUs; no reference counterpart -- the
 * reference runs every unit on one GPU).  After this call ocean_step computes the
 * full row IFFT of every row (the rows are needed whole) but stores, column-transforms
 * and fills only the columns x_begin <= x < x_begin + x_count of every slice: DISP,
 * DERIV, TURB and NORMAL are written there, bit-identical to a whole-band context's
 * texels, and the other columns are left as they are (zero after ocean_create).
 * Two contexts with complementary bands (one per GPU) produce a cascade between them
 * with no data exchange.  x_begin and x_count are multiples of g = min(N, max(16,
 * 8192 / N)); (0, N) restores the whole band.  Needs the fused schedule (not
 * OCEAN_F_UNFUSED) and no OCEAN_F_MIPS; the unfused stages (ocean_evolve,
 * ocean_ifft2d, ocean_fill) ignore the band. */
int ocean_set_column_band(ocean_ctx *ctx, int x_begin, int x_count);

/* Column parity, the other way to split one unit over two GPUs (no reference
 * counterpart): with parity b in {0, 1} the context computes only the output columns x = 2m + b,
 * m < N/2, of every slice, by decimation in frequency of the row transform (each row is evolved
 * whole, folded to z_b[n] = (a[n] + (-1)^b a[n + N/2]) e^{2 pi i b n / N} and transformed at N/2
 * points), so the two ranks of a unit do not duplicate the row transform as column bands do.
 * Column x = 2m + b is stored COMPACT at texture column m (DISP, DERIV, TURB, NORMAL: the first
 * N/2 columns of each texture row; the rest are left as they are); the consumer interleaves the
 * two ranks' textures.  Results equal the whole context's within the fp32 tolerance (a different
 * radix order), not bit for bit.  N = 4096, fused full-output schedule, no OCEAN_F_MIPS; -1 turns
 * it off (whole band again).  ocean_set_column_band replaces a parity; world sampling of a parity
 * context returns OCEAN_E_UNSUPPORTED. */
int ocean_set_column_parity(ocean_ctx *ctx, int parity);

/* Replaces the TimeDependentSpectrum dispatch alone (WaterBody.cs:181-182;
 * TimeDependentSpectrum.compute:20-47): writes PLANE0..3 at `time`.  Async. */
int ocean_evolve(ocean_ctx *ctx, float time);

/* Replaces IFFT.InverseFastFourierTransform(RenderTexture) (IFFT.cs:66-94) for
 * every plane p with bit p set in `plane_mask`: in place,
 * out[m] = (-1)^(mx+my) * sum_{x,y} in[x,y] e^{+2 pi i (x mx + y my)/N}
 * over all tiles and cascades.  Async. */
int ocean_ifft2d(ocean_ctx *ctx, int plane_mask);

/* Replaces the FillResultTextures dispatch (WaterBody.cs:189;
 * ResultTexturesFiller.compute:16-34): PLANE0..3 + TURB -> DISP, DERIV, TURB.  Async. */
int ocean_fill(ocean_ctx *ctx);

/* Synchronous texture readback of one (tile, cascade) slice, replacing
 * AsyncGPUReadback.Request(...).GetData<Color>() (WaterBody.cs:288-296).
 * `bytes` must equal the slice size (N*N*16 for float4, N*N*8 for float2).
 * Orders after all work queued on the ctx stream. */
int ocean_read(ocean_ctx *ctx, int texture, int tile, int cascade, void *dst, size_t bytes);

/* Synchronous upload of one slice (foam state for resume, planes for
 * operator-level tests).  Same size rules as ocean_read.  OCEAN_TEX_WAVES is
 * writable only with OCEAN_F_UNFUSED (E_UNSUPPORTED otherwise): the fused row pass
 * rebuilds the wave data from the active parameters every frame. */
int ocean_write(ocean_ctx *ctx, int texture, int tile, int cascade, const void *src, size_t bytes);

/* Zero-copy access for same-process consumers: base device pointer and total
 * byte size of a texture (all tiles and cascades). */
int ocean_get_device_ptr(ocean_ctx *ctx, int texture, void **ptr, size_t *bytes);

/* The ctx's hipStream_t (as void*), for callers that order their own work. */
int ocean_get_stream(ocean_ctx *ctx, void **stream);

/* Blocks until all work queued on the ctx stream has finished. */
int ocean_synchronize(ocean_ctx *ctx);

/* Kernel timing: when enabled, each kernel launch of ocean_step / ocean_ifft2d
 * is bracketed by HIP events on the ctx stream; ocean_kernel_stats returns, for
 * kernel `kind` (0 = pass A / row pass, 1 = pass B / column pass, 2 = other),
 * the summed duration in ms and the launch count since the last reset
 * (synchronizes the stream).  At most 2048 launches' events are held: past that
 * the finished ones are folded into the sums (waiting for the oldest if none
 * has finished), and disabling timing folds the rest, so a host that never
 * polls holds a bounded number of events. */
int ocean_set_kernel_timing(ocean_ctx *ctx, int enable);
int ocean_kernel_stats(ocean_ctx *ctx, int kind, double *total_ms, long long *launches);

/* Symbol (demangled, as rocprofv3 reports it) of the kernel most recently launched in `kind`
 * (0, 1, 2 as above) by this context, NUL-terminated into buf[len].  OCEAN_E_STATE if none yet;
 * OCEAN_E_INVALID_ARG if it does not fit.  Measurement only (no reference counterpart): lets a
 * bench match profiler records to the exact kernel that ran. */
int ocean_kernel_name(ocean_ctx *ctx, int kind, char *buf, size_t len);

/* Algorithmic HBM bytes one ocean_step moves in the schedule this context runs
 * (the roofline numerator; no reference counterpart -- measurement only):
 * fused: *pass_a = pass A (evolve + row IFFT), *pass_b = pass B (column IFFT +
 * fill); OCEAN_F_UNFUSED: *pass_a = evolve + row launches, *pass_b = column
 * launches + fill.  Depends on the kernels selected for N, the flags and the
 * state (e.g. after ocean_write(H0) pass A reads the full h0). */
int ocean_step_bytes(ocean_ctx *ctx, uint64_t *pass_a, uint64_t *pass_b);

/* Mip chains (OCEAN_F_MIPS), the GenerateMips of WaterBody.cs:191-192.  Level
 * L >= 1 of a slice is (N >> L)^2 RGBA fp32 texels, [y][x]; texel (x, y) =
 * ((a + b) + (c + d)) * 0.25 over the 2x2 texels (2x, 2y), (2x+1, 2y),
 * (2x, 2y+1), (2x+1, 2y+1) of level L-1 (a box filter: Unity's filter is not
 * specified).  Level 0 is the texture itself.  `texture` is OCEAN_TEX_DERIV or
 * OCEAN_TEX_TURB; bytes must equal (N >> level)^2 * 16.  Blocking, like ocean_read.
 * Device layout (ocean_get_mip_ptr): one chain per slice, levels 1..log2 N
 * concatenated, slice-major; *ptr points at level `level` of slice 0 and
 * *slice_stride is the distance in bytes between consecutive slices' chains. */
int ocean_read_mip(ocean_ctx *ctx, int texture, int tile, int cascade, int level, void *dst, size_t bytes);
int ocean_get_mip_ptr(ocean_ctx *ctx, int texture, int level, void **ptr, size_t *slice_stride);

/* Cascade-summed world sampling, the texture reads of the reference's consumer
 * (Water.shader:314-348).  Point i of `points` is (world x,
 * world z, lod) as float[3]; out[i] is float[12]:
 *   out[12i + 0..3]  = sum_c DISP_c(uv_c).xyz, sum_c (1 - saturate(TURB_c(uv_c, lod).x))
 *   out[12i + 4..7]  = sum_c DERIV_c(uv_c, lod)            (Dyx, Dyz, Dxx, Dzz)
 *   out[12i + 8..11] = normalize(-sx, 1, -sz), 0 with s = (d.x / (1 + d.z), d.y / (1 + d.w))
 * over the cascades c of tile `tile`, uv_c = (x, z) / L_c (L_c = the active cascade
 * wavelength), summed in cascade order from 0.  Filtering (this library's definition;
 * Unity's RenderTextures are Repeat-wrapped and trilinear, WaterBody.cs:112-113):
 * on an m x m level, s = uv * m - 0.5, texels floor(s) and floor(s) + 1 mod m, weights
 * f = s - floor(s), lerp(a, b, f) = a + f (b - a), x first then y.  DISP has no mips
 * (WaterBody.cs:227) and is read at level 0; DERIV and TURB blend levels floor(lod)
 * and floor(lod) + 1 (lod clamped to [0, log2 N]) when the context has OCEAN_F_MIPS,
 * else level 0.  DISPLACEMENT_ONLY contexts return zero derivatives and turbulence.
 * ocean_sample_world takes host buffers and blocks; ocean_sample_world_device takes
 * device pointers (points 4-B aligned, out 16-B aligned, else OCEAN_E_INVALID_ARG) and
 * is async on the ctx stream, ordered after the queued steps.  count = 0 is a no-op.
 * Both return OCEAN_E_STATE before ocean_init_spectrum. */
int ocean_sample_world(ocean_ctx *ctx, int tile, const float *points, int count, float *out);
int ocean_sample_world_device(ocean_ctx *ctx, int tile, const float *points, int count, float *out);

/* Asynchronous readback, the AsyncGPUReadback.Request(tex, 0, callback) of
 * WaterBody.cs:288-296: copies one slice (level 0) to `dst` on a copy stream once
 * the work queued so far on the ctx stream (e.g. the last ocean_step) has finished,
 * without blocking the caller.  `dst` must stay valid until the request is done;
 * for a truly asynchronous copy it should come from ocean_host_alloc (pinned).
 * ocean_readback_status: 1 done, 0 pending, < 0 error (the request's hasError).
 * ocean_readback_wait blocks until done.  Every request is freed with
 * ocean_readback_release (after completion; releasing a pending request waits). */
typedef struct ocean_readback ocean_readback;
int ocean_read_async(ocean_ctx *ctx, int texture, int tile, int cascade, void *dst, size_t bytes,
                     ocean_readback **out);
int ocean_readback_status(ocean_readback *rb);
int ocean_readback_wait(ocean_readback *rb);
void ocean_readback_release(ocean_readback *rb);
/* Height-only readback for buoyancy: the reference reads displacement slice 0 back every frame
 * (WaterBody.cs:288-296) into its private buoyancyData (:58), whose only reader, GetWaterHeight,
 * returns the .g channel alone (:195-209).  This request copies just that channel, DISP.y = Dy of one
 * (tile, cascade) slice, as float[N][N] laid out [y][x] (`bytes` = N*N*4: a quarter of the RGBA
 * slice over the link), with ocean_read_async's snapshot and completion semantics: the same
 * ocean_readback_status / _wait / _release / _copy_ms apply.  dst[y*N + x] is bit-identical to
 * the .y of texel (x, y) of the RGBA slice read at the same point of the stream. */
int ocean_read_height_async(ocean_ctx *ctx, int tile, int cascade, float *dst, size_t bytes,
                            ocean_readback **out);

/* Readback timing (off after ocean_create): while on, each new ocean_read_async /
 * ocean_read_height_async request records HIP timing events around its device-to-host copy, for
 * ocean_readback_copy_ms.  Requests made while it is off record only untimed events. */
int ocean_set_readback_timing(ocean_ctx *ctx, int enable);

/* Duration of a completed request's device-to-host copy in ms (HIP events on the copy stream around
 * the copy itself: the link's share of the request, without the wait for the queued frames or the
 * on-device snapshot).  OCEAN_E_STATE while the request is pending, or if it was made with readback
 * timing off.  No reference counterpart: AsyncGPUReadback exposes no timing; hosts use it to
 * attribute a readback-bound loop. */
int ocean_readback_copy_ms(ocean_readback *rb, float *ms);

/* Pinned host memory for ocean_read_async destinations (hipHostMalloc). */
int ocean_host_alloc(size_t bytes, void **out);
void ocean_host_free(void *p);

/* Thread-local message describing the last failure on this thread ("" if none). */
const char *ocean_last_error(void);

/* OCEAN_ABI_VERSION of the loaded library. */
int ocean_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* OCEAN_OCEAN_H */
