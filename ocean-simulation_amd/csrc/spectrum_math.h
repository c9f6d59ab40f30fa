// Per-texel spectrum arithmetic shared by the elementwise kernels (spectrum.hip)
// and the fused row passes (fft3.hip).  Every expression keeps the
// reference's fp32 operation order; the library is built with
// -ffp-contract=off so no FMA contraction changes a rounding (the phase
// omega*t at large t is sensitive to one ulp of omega).
#pragma once

#include <hip/hip_runtime.h>

namespace ocean {

constexpr float kPi = 3.14159265f;                         // InitialSpectrum.compute:8
constexpr float kFoamDecay = 0.135335283236612691894f;     // exp(-2), ResultTexturesFiller.compute:29-30

struct Planes4 {
    float2 p[4];  // DxDz, DyDxz, DyxDyz, DxxDzz
};

// Wave data of texel (x, y) of a cascade (InitialSpectrum.compute:101-126):
// k = (nx, nz) * dk, dk = 2 pi / L; in band [lo, hi]: (kx, 1/|k|, kz,
// omega = sqrt(g |k|)), else (kx, 1, kz, 0).  Used by the init kernel AND
// recomputed per frame by the fused row pass, so both see bit-identical values
// (only correctly rounded + - * / sqrt).
struct WaveBand {
    float dk, lo, hi;
};

// `cs` = {L, cutoff_low, cutoff_high, ...} (ocean_cascade order).
__device__ __forceinline__ WaveBand wave_band(const float* cs) {
    return WaveBand{2.0f * kPi / cs[0], cs[1], cs[2]};  // :110
}

__device__ __forceinline__ float4 wave_data(int x, int y, int n, WaveBand b, float g, float* kmag_out = nullptr) {
    const int nx = x - n / 2, nz = y - n / 2;
    const float kx = (float)nx * b.dk, kz = (float)nz * b.dk;
    const float kmag = sqrtf(kx * kx + kz * kz);
    if (kmag_out) *kmag_out = kmag;
    if (kmag >= b.lo && kmag <= b.hi) return make_float4(kx, 1.0f / kmag, kz, sqrtf(g * kmag));
    return make_float4(kx, 1.0f, kz, 0.0f);
}

// sin and cos of an fp32 argument, |x| < 2^17 on the fast path: Cody-Waite
// reduction by pi/2 with a three-part FMA split (exact products), then
// minimax polynomials on [-pi/4, pi/4] (Cephes sinf/cosf coefficients);
// max error ~1-2 ulp against correctly rounded sin/cos.  Larger |x| falls back
// to the library sincosf.  ~25 VALU instead of the library's ~45 plus its
// Payne-Hanek branch.
__device__ __forceinline__ void sincos_fast(float x, float* s, float* c) {
    if (!(fabsf(x) < 131072.0f)) {
        sincosf(x, s, c);
        return;
    }
    const float n = rintf(x * 0.636619772367581343f);
    float r = fmaf(-n, 1.57079637050628662109375f, x);
    r = fmaf(-n, -4.37113882867379e-08f, r);
    r = fmaf(-n, -1.7151245e-15f, r);
    const float r2 = r * r;
    const float sp = fmaf(fmaf(fmaf(-1.9515295891e-4f, r2, 8.3321608736e-3f), r2, -1.6666654611e-1f), r2 * r, r);
    const float cp = fmaf(fmaf(fmaf(2.443315711809948e-5f, r2, -1.388731625493765e-3f), r2, 4.166664568298827e-2f),
                          r2 * r2, fmaf(-0.5f, r2, 1.0f));
    const int q = (int)n & 3;
    const float ss = (q & 1) ? cp : sp, cc = (q & 1) ? sp : cp;
    *s = (q & 2) ? -ss : ss;
    *c = ((q + 1) & 2) ? -cc : cc;
}

// TimeDependentSpectrum.compute:20-47 for one texel-cascade, split in the
// phase factor e = exp(i omega t) (:25, shared by k and its mirror -k, which
// have the same |k| and so the same omega) and the per-texel products.
struct Phase {
    float ex, ey;
};
__device__ __forceinline__ Phase evolve_phase(float omega, float t) {
    Phase e;
    sincos_fast(omega * t, &e.ey, &e.ex);
    return e;
}
// h(k, t) = ComplexMult(h0.xy, e) + ComplexMult(h0.zw, conj(e))  (:26)
__device__ __forceinline__ float2 evolve_h(float4 h, Phase e) {
    const float ex = e.ex, ey = e.ey;
    return make_float2((h.x * ex - h.y * ey) + (h.z * ex - h.w * (-ey)), (h.x * ey + h.y * ex) + (h.z * (-ey) + h.w * ex));
}
// The four packed planes of one texel from h(k, t) and its wave data (:27-45).
__device__ __forceinline__ Planes4 planes_of(float2 h, float4 w) {
    Planes4 o;
    const float hx = h.x, hy = h.y;
    float ihx = -hy, ihy = hx;                                   // :27
    float ydx_x = ihx * w.x, ydx_y = ihy * w.x;                  // :29
    float ydz_x = ihx * w.z, ydz_y = ihy * w.z;                  // :30
    float dx_x = ydx_x * w.y, dx_y = ydx_y * w.y;                // :32
    float dz_x = ydz_x * w.y, dz_y = ydz_y * w.y;                // :34
    float aux_x = -hx * w.y, aux_y = -hy * w.y;                  // :36
    float dxdx_x = aux_x * w.x * w.x, dxdx_y = aux_y * w.x * w.x;  // :38
    float dzdz_x = aux_x * w.z * w.z, dzdz_y = aux_y * w.z * w.z;  // :39
    float dzdx_x = aux_x * w.x * w.z, dzdx_y = aux_y * w.x * w.z;  // :40
    o.p[0] = make_float2(dx_x - dz_y, dx_y + dz_x);              // :42 DxDz
    o.p[1] = make_float2(hx - dzdx_y, hy + dzdx_x);              // :43 DyDxz
    o.p[2] = make_float2(ydx_x - ydz_y, ydx_y + ydz_x);          // :44 DyxDyz
    o.p[3] = make_float2(dxdx_x - dzdz_y, dxdx_y + dzdz_x);      // :45 DxxDzz
    return o;
}
__device__ __forceinline__ Planes4 evolve_with(float4 h, float4 w, Phase e) { return planes_of(evolve_h(h, e), w); }
__device__ __forceinline__ Planes4 evolve_texel(float4 h, float4 w, float t) {
    return evolve_with(h, w, evolve_phase(w.w, t));
}

// ResultTexturesFiller.compute:27-32: Jacobian and the foam accumulator.
__device__ __forceinline__ float foam_update(float prev, float dxx, float dzz, float dxz) {
    float jac = (1.0f + dxx) * (1.0f + dzz) - dxz * dxz;
    float foam = prev * kFoamDecay;
    if (foam < jac) foam += jac;
    return foam;
}

// Derived per-cascade normal (Water.shader:346-348 applied to one cascade's derivatives).
__device__ __forceinline__ float4 normal_from_deriv(float dyx, float dyz, float dxx, float dzz) {
    float sx = dyx / (1.0f + dxx);
    float sz = dyz / (1.0f + dzz);
    float inv = 1.0f / sqrtf(sx * sx + 1.0f + sz * sz);
    return make_float4(-sx * inv, inv, -sz * inv, 0.0f);
}

}  // namespace ocean
