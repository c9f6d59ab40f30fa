// World sampling of the texture-out contract (ocean_sample_world).
//
// The reference's consumer, Water.shader, reads the cascade textures at world
// positions: the Domain stage sums the displacement of every cascade sampled at
// uv = worldXZ / _Wavelengths[i] (:320-326), the Fragment stage sums derivatives and
// 1 - saturate(turbulence.x) the same way (:338-344) and builds the normal from the
// summed derivatives (:346-347).  The RenderTextures are Repeat-wrapped and
// trilinear-filtered (WaterBody.cs:112-113); the displacement array has no mips
// (:227), derivatives and turbulence do (:228-229).
//
// One lane per query point.  Filtering is stated exactly (the GPU's texture units
// round their weights in ways Unity does not specify, so this is this library's
// definition, restated in fp32 by oracle.sample_world):
//   level texture of side m, uv = (x / L, z / L):  sx = u * m - 0.5, sy = v * m - 0.5;
//   i = floor(s), f = s - floor(s); texel columns i mod m, i + 1 mod m (Repeat), rows alike;
//   bilinear = lerp(lerp(t00, t10, fx), lerp(t01, t11, fx), fy), lerp(a, b, f) = a + f (b - a);
//   trilinear (DERIV, TURB with OCEAN_F_MIPS): lod clamped to [0, log2 N],
//   lerp(level floor(lod), level floor(lod) + 1, lod - floor(lod)); without mip chains
//   and for DISP, level 0.
// Random gathers of 4-16 texels per cascade: L2 / Infinity-Cache latency bound, not
// part of the frame (no roofline claimed).
#include "ocean_internal.h"
#include "spectrum_math.h"

namespace ocean {
namespace {

struct Bil {
    int x0, x1, y0, y1;
    float fx, fy;
};

// Texel coordinates + weights of a bilinear tap at uv on an m x m level (m a power
// of two).  floor(s) is wrapped exactly in float (integers, power-of-two scaling),
// so any finite uv works without integer overflow.
__device__ __forceinline__ Bil bil(float u, float v, int m) {
    const float fm = (float)m, inv = 1.0f / fm;
    const float sx = u * fm - 0.5f, sy = v * fm - 0.5f;
    const float flx = floorf(sx), fly = floorf(sy);
    Bil b;
    b.fx = sx - flx;
    b.fy = sy - fly;
    const int ix = (int)(flx - fm * floorf(flx * inv)), iy = (int)(fly - fm * floorf(fly * inv));
    b.x0 = ix;
    b.x1 = (ix + 1) & (m - 1);
    b.y0 = iy;
    b.y1 = (iy + 1) & (m - 1);
    return b;
}

__device__ __forceinline__ float4 lerp4(float4 a, float4 b, float f) {
    return make_float4(a.x + f * (b.x - a.x), a.y + f * (b.y - a.y), a.z + f * (b.z - a.z), a.w + f * (b.w - a.w));
}

__device__ __forceinline__ float4 add4(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__device__ __forceinline__ float4 tap(const float4* __restrict__ t, int m, const Bil& b) {
    const float4 t00 = t[(size_t)b.y0 * m + b.x0], t10 = t[(size_t)b.y0 * m + b.x1];
    const float4 t01 = t[(size_t)b.y1 * m + b.x0], t11 = t[(size_t)b.y1 * m + b.x1];
    return lerp4(lerp4(t00, t10, b.fx), lerp4(t01, t11, b.fx), b.fy);
}

// Level l of a slice: level 0 is the texture slice, levels >= 1 come from its mip chain.
__device__ __forceinline__ const float4* level_ptr(const float4* tex0, const float4* chain, size_t chain_len,
                                                   int slice, int n, int l) {
    if (l == 0) return tex0 + (size_t)slice * n * n;
    size_t off = 0;
    for (int k = 1; k < l; ++k) off += (size_t)(n >> k) * (n >> k);
    return chain + (size_t)slice * chain_len + off;
}

__device__ __forceinline__ float4 tri(const float4* tex0, const float4* chain, size_t chain_len, int slice, int n,
                                      int logn, float u, float v, float lod) {
    if (!chain || !(lod > 0.0f)) return tap(tex0 + (size_t)slice * n * n, n, bil(u, v, n));
    const float lc = fminf(lod, (float)logn);
    const int l0 = (int)floorf(lc), l1 = min(l0 + 1, logn);
    const float f = lc - (float)l0;
    const int m0 = n >> l0, m1 = n >> l1;
    const float4 a = tap(level_ptr(tex0, chain, chain_len, slice, n, l0), m0, bil(u, v, m0));
    const float4 b = tap(level_ptr(tex0, chain, chain_len, slice, n, l1), m1, bil(u, v, m1));
    return lerp4(a, b, f);
}

// Point i: (world x, world z, lod) -> out[i] = {(Dx, Dy, Dz, turbulence), (Dyx, Dyz, Dxx, Dzz), normal}.
__global__ __launch_bounds__(256) void k_sample_world(DevView v, int tile, const float* __restrict__ pts, int count,
                                                      float4* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const float x = pts[3 * (size_t)i], z = pts[3 * (size_t)i + 1], lod = pts[3 * (size_t)i + 2];
    float4 disp = make_float4(0.0f, 0.0f, 0.0f, 0.0f), deriv = disp;
    float turb = 0.0f;
    for (int c = 0; c < v.C; ++c) {
        const float L = v.casc[c * 5];
        const float u = x / L, w = z / L;  // worldUV / _Wavelengths[i] (Water.shader:325, :341)
        const int slice = tile * v.C + c;
        disp = add4(disp, tap(v.disp + (size_t)slice * v.n * v.n, v.n, bil(u, w, v.n)));  // no mips (:325)
        if (v.deriv) {
            deriv = add4(deriv, tri(v.deriv, v.deriv_mips, v.mip_chain, slice, v.n, v.logn, u, w, lod));
            const float tb = tri(v.turb, v.turb_mips, v.mip_chain, slice, v.n, v.logn, u, w, lod).x;
            turb = turb + (1.0f - fminf(fmaxf(tb, 0.0f), 1.0f));  // 1 - saturate(.x) (:343)
        }
    }
    out[3 * (size_t)i] = make_float4(disp.x, disp.y, disp.z, turb);
    out[3 * (size_t)i + 1] = deriv;
    out[3 * (size_t)i + 2] = normal_from_deriv(deriv.x, deriv.y, deriv.z, deriv.w);  // :346-347
}

}  // namespace

hipError_t launch_sample_world(const DevView& v, int tile, const float* pts, int count, float* out, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    const unsigned g = (unsigned)((count + 255) / 256);
    launch(k_sample_world, dim3(g), dim3(256), 0, s, v, tile, pts, count, reinterpret_cast<float4*>(out));
    return hipGetLastError();
}

}  // namespace ocean
