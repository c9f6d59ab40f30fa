// Spectrum kernels for gfx950: initial spectrum (+ Hermitian partner),
// unfused evolve and unfused fill.  One thread per texel, 16-byte vector loads
// and stores, grid-strided over every (tile, cascade) unit.
//
//   init_spectrum   InitialSpectrum.compute:33-129
//   conjugate       InitialSpectrum.compute:135-143 (out of place: h0 -> h0)
//   evolve          TimeDependentSpectrum.compute:20-47
//   fill            ResultTexturesFiller.compute:16-34
#include "ocean_internal.h"
#include "spectrum_math.h"

namespace ocean {
namespace {

// ---------------- InitialSpectrum.compute helpers (:33-97) -----------------
struct Sp {
    float U, g, F, D, wdx, wdy;
};

// AngularFrequency (:33-35) = sqrt(g |k|) lives in wave_data (spectrum_math.h).

// The transcendentals of the initial spectrum, each correctly rounded: evaluated in double and rounded
// once to fp32, as the oracle does (oracle/ocean_oracle.c cr_*), so h0 is bit-exact between the two.
// The device's fp32 powf / expf / atan2f / ... differed from it in 63-72 % of h0 texels by a few ulp,
// and that difference was the whole of the library's pointwise excess over the oracle's own fp32 error
// (2.5-3.0x, tools/pointwise_stages.py, docs/MEASUREMENTS.md section 9).  Runs once per init.
__device__ __forceinline__ float sp_pow(float a, float b) { return (float)pow((double)a, (double)b); }
__device__ __forceinline__ float sp_exp(float a) { return (float)exp((double)a); }
__device__ __forceinline__ float sp_log(float a) { return (float)log((double)a); }
__device__ __forceinline__ float sp_tanh(float a) { return (float)tanh((double)a); }
__device__ __forceinline__ float sp_cosh(float a) { return (float)cosh((double)a); }
__device__ __forceinline__ float sp_cos(float a) { return (float)cos((double)a); }
__device__ __forceinline__ float sp_atan2(float a, float b) { return (float)atan2((double)a, (double)b); }

__device__ __forceinline__ float tma_correction(const Sp& p, float w) {  // :38-43
    float wh = w * sqrtf(p.D / p.g);
    if (wh <= 1.0f) return 0.5f * wh * wh;
    if (wh < 2.0f) return 1.0f - 0.5f * (2.0f - wh) * (2.0f - wh);
    return 1.0f;
}

__device__ __forceinline__ float jonswap(const Sp& p, float w, float wp) {  // :47-56
    float alpha = 0.076f * sp_pow(fabsf(p.U * p.U / (p.F * p.g)), 0.22f);
    float gamma = 3.3f;
    float sigma = w <= wp ? 0.07f : 0.09f;
    float d = w - wp;
    float r = sp_exp(-(d * d) / (2.0f * sigma * sigma * wp * wp));
    return alpha * p.g * p.g / sp_pow(w, 5.0f) * sp_exp(-1.25f * sp_pow(wp / w, 4.0f)) * sp_pow(fabsf(gamma), r);
}

__device__ __forceinline__ float spread_power(const Sp& p, float w, float wp) {  // :60-66
    if (w < 1.05f * wp) return 6.97f * sp_pow(fabsf(w / wp), 4.06f);
    float peak_speed = p.g / wp;
    float mu = -2.33f - 1.45f * (p.U / peak_speed - 1.17f);
    return 9.77f * sp_pow(fabsf(w / wp), mu);
}

__device__ __forceinline__ float normalization_factor(float s) {  // :69-74
    float s2 = s * s;
    float s3 = s2 * s;
    if (s <= 0.4f)
        return 0.09f * s3 + (sp_pow(sp_log(2.0f), 2.0f) / kPi - kPi / 12.0f) * s2 + sp_log(2.0f) / kPi * s +
               1.0f / (2.0f * kPi);
    return sqrtf(s) / (2.0f * sqrtf(kPi)) + 1.0f / (16.0f * sqrtf(kPi * s));
}

__device__ __forceinline__ float directional_spread(const Sp& p, float w, float wp, float theta, float swell) {  // :78-84
    float s = spread_power(p, w, wp) + 16.0f * sp_tanh(w / wp) * swell * swell;
    float len = sqrtf(p.wdx * p.wdx + p.wdy * p.wdy);  // normalize(float2(x, y))
    float wind_theta = sp_atan2(p.wdy / len, p.wdx / len);
    return normalization_factor(s) * sp_pow(fabsf(sp_cos(0.5f * (theta - wind_theta))), 2.0f * s);
}

__device__ __forceinline__ float frequency_derivative(const Sp& p, float k, float w) {  // :87-91
    float th = sp_tanh(fminf(k * p.D, 20.0f));
    float ch = sp_cosh(k * p.D);
    return p.g * (p.D * k / ch / ch + th) / (w * 2.0f);
}

__device__ __forceinline__ float short_waves_fade(float k, float fade) { return sp_exp(-fade * fade * k * k); }  // :95-97

// CalculateInitialSpectrumTextures (:99-129): one thread per (unit, texel).
__global__ __launch_bounds__(256) void k_init_spectrum(DevView v, Sp p) {
    const int n = v.n;
    const size_t plane = (size_t)n * n;
    const size_t total = plane * v.units;
    const float wp = 22.0f * sp_pow(fabsf(p.g * p.g / (p.U * p.F)), 0.3333f);  // :118
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int u = (int)(i / plane);
        const size_t t = i - (size_t)u * plane;
        const int y = (int)(t / n), x = (int)(t - (size_t)y * n);
        const int tile = u / v.C, c = u - tile * v.C;
        const float* cs = v.casc + c * 5;
        const float2 g = v.noise[(size_t)tile * plane + t];
        const float dk = 2.0f * kPi / cs[0];  // :110
        float kmag;
        const float4 w = wave_data(x, y, n, wave_band(cs), p.g, &kmag);
        float4 h;
        if (kmag >= cs[1] && kmag <= cs[2]) {  // :114
            const float kangle = sp_atan2(w.z, w.x);
            const float om = w.w;  // angular_frequency(kmag) (:116), computed in wave_data
            const float amp = sqrtf(2.0f * tma_correction(p, om) * jonswap(p, om, wp) *
                                    directional_spread(p, om, wp, kangle, cs[3]) * short_waves_fade(kmag, cs[4]) *
                                    frequency_derivative(p, kmag, om) / kmag * dk * dk);
            h = make_float4(g.x / 2.0f * amp, g.y / 2.0f * amp, 0.0f, 0.0f);
        } else {
            h = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
        v.h0[i] = h;
        if (v.h0k) v.h0k[i] = make_float2(h.x, h.y);
        v.waves[i] = w;
    }
}

// CalculateConjugatedInitialSpectrumTextures (:135-143).  h0.xy is never
// modified by this pass, so reading the mirror's .xy while other threads
// rewrite their texel is race-free when .xy is written unchanged; we still
// only store .zw lanes' new values alongside the unchanged .xy.
__global__ __launch_bounds__(256) void k_conjugate(DevView v) {
    const int n = v.n;
    const size_t plane = (size_t)n * n;
    const size_t total = plane * v.units;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int u = (int)(i / plane);
        const size_t t = i - (size_t)u * plane;
        const int y = (int)(t / n), x = (int)(t - (size_t)y * n);
        const int mx = (n - x) & (n - 1), my = (n - y) & (n - 1);
        const float4* src = v.h0 + (size_t)u * plane;
        const float2 hk = *reinterpret_cast<const float2*>(&src[t]);
        const float2 hm = *reinterpret_cast<const float2*>(&src[(size_t)my * n + mx]);
        // write only .zw: .xy stays as is (no writer/reader conflict on .xy)
        float2* dst = reinterpret_cast<float2*>(&v.h0[i]) + 1;
        *dst = make_float2(hm.x, -hm.y);
        (void)hk;
    }
}

__global__ __launch_bounds__(256) void k_evolve(DevView v, float time) {
    const size_t total = (size_t)v.n * v.n * v.units;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        Planes4 o = evolve_texel(v.h0[i], v.waves[i], time);
        for (int p = 0; p < v.planes; ++p) v.plane[p][i] = o.p[p];
    }
}

// Index of texel i = (u, y, x) in the column-tile-major layout [u][x/W][y][W]
// of the foam state (and of the fused path's intermediate planes).
__device__ __forceinline__ size_t tiled_index(size_t i, int n, int w) {
    const size_t plane = (size_t)n * n;
    const size_t u = i / plane, t = i - u * plane;
    const int y = (int)(t / n), x = (int)(t - (size_t)y * n);
    return ((u * (n / w) + x / w) * n + y) * w + (x % w);
}

__global__ __launch_bounds__(256) void k_fill(DevView v) {
    const size_t total = (size_t)v.n * v.n * v.units;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const float2 a = v.plane[0][i], b = v.plane[1][i];
        v.disp[i] = make_float4(a.x, b.x, a.y, 1.0f);
        if (v.planes == 4) {
            const float2 c = v.plane[2][i], d = v.plane[3][i];
            v.deriv[i] = make_float4(c.x, c.y, d.x, d.y);
            const size_t fi = tiled_index(i, v.n, v.tile_w);
            const float foam = foam_update(v.foam[fi], d.x, d.y, b.y);
            v.foam[fi] = foam;
            v.turb[i] = make_float4(foam, foam, foam, foam);
            if (v.normals) v.normal[i] = normal_from_deriv(c.x, c.y, d.x, d.y);
        }
    }
}

// Foam state <- TURB.x (after an ocean_write of the TURB texture: resume).
__global__ __launch_bounds__(256) void k_foam_import(DevView v) {
    const size_t total = (size_t)v.n * v.n * v.units;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
        v.foam[tiled_index(i, v.n, v.tile_w)] = v.turb[i].x;
}

// Device noise (ocean_generate_noise_device): a counter-based stream per texel so
// every texel is independent work.  Texel (x, y) of tile t draws its k-th uniform
// from h_k = mix(key + (k + 1) * 0x9E3779B97F4A7C15), key = mix(seed + t) ^ (y * N + x)
// * 0xD1B54A32D192ED03 (mix = the splitmix64 finaliser), U = (h_k >> 40) * 2^-24,
// and each of g1, g2 comes from the reference's Marsaglia polar loop
// (WaterBody.cs:71-81: v = 2U - 1, reject s >= 1 or s == 0, keep v1 sqrt(-2 ln s / s)).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_noise(float2* __restrict__ noise, int n, int tiles, uint64_t seed) {
    const size_t plane = (size_t)n * n;
    const size_t total = plane * tiles;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t t = i / plane, texel = i - t * plane;
        const uint64_t key = mix64(seed + t + 0x9E3779B97F4A7C15ull) ^ (texel * 0xD1B54A32D192ED03ull);
        uint64_t k = 0;
        auto uniform = [&]() {
            ++k;
            return (float)(mix64(key + k * 0x9E3779B97F4A7C15ull) >> 40) * (1.0f / 16777216.0f);
        };
        float g[2];
        for (int c = 0; c < 2; ++c) {
            float v1, v2, q;
            do {
                v1 = 2.0f * uniform() - 1.0f;
                v2 = 2.0f * uniform() - 1.0f;
                q = v1 * v1 + v2 * v2;
            } while (q >= 1.0f || q == 0.0f);
            g[c] = v1 * sqrtf(-2.0f * logf(q) / q);
        }
        noise[i] = make_float2(g[0], g[1]);
    }
}

// h0k <- h0.xy (ocean_set_column_parity allocates h0k for pass A3PP after the spectrum may exist)
__global__ __launch_bounds__(256) void k_h0k_extract(DevView v) {
    const size_t total = (size_t)v.n * v.n * v.units;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
        v.h0k[i] = *reinterpret_cast<const float2*>(&v.h0[i]);
}

unsigned grid_for(size_t total) {
    size_t g = (total + 255) / 256;
    return (unsigned)(g < 16384 ? (g == 0 ? 1 : g) : 16384);
}

}  // namespace

hipError_t launch_noise(const DevView& v, uint64_t seed, hipStream_t s) {
    const size_t total = (size_t)v.n * v.n * v.T;
    launch(k_noise, dim3(grid_for(total)), dim3(256), 0, s, const_cast<float2*>(v.noise), v.n, v.T, seed);
    return hipGetLastError();
}

hipError_t launch_init_spectrum(const DevView& v, const SpectrumParams& sp, hipStream_t s) {
    Sp p{sp.wind_speed, sp.gravity, sp.fetch, sp.depth, sp.wind_dir_x, sp.wind_dir_y};
    launch(k_init_spectrum, dim3(grid_for((size_t)v.n * v.n * v.units)), dim3(256), 0, s, v, p);
    return hipGetLastError();
}

hipError_t launch_conjugate(const DevView& v, hipStream_t s) {
    launch(k_conjugate, dim3(grid_for((size_t)v.n * v.n * v.units)), dim3(256), 0, s, v);
    return hipGetLastError();
}

hipError_t launch_evolve(const DevView& v, float t, hipStream_t s) {
    launch(k_evolve, dim3(grid_for((size_t)v.n * v.n * v.units)), dim3(256), 0, s, v, t);
    return hipGetLastError();
}

hipError_t launch_foam_import(const DevView& v, hipStream_t s) {
    launch(k_foam_import, dim3(grid_for((size_t)v.n * v.n * v.units)), dim3(256), 0, s, v);
    return hipGetLastError();
}

hipError_t launch_h0k_extract(const DevView& v, hipStream_t s) {
    if (!v.h0k) return hipErrorInvalidValue;
    launch(k_h0k_extract, dim3(grid_for((size_t)v.n * v.n * v.units)), dim3(256), 0, s, v);
    return hipGetLastError();
}

hipError_t launch_fill(const DevView& v, hipStream_t s) {
    launch(k_fill, dim3(grid_for((size_t)v.n * v.n * v.units)), dim3(256), 0, s, v);
    return hipGetLastError();
}

}  // namespace ocean
