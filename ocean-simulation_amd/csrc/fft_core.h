// Shared FFT building blocks for gfx950: in-register inverse DFTs of radix
// 2/4/8/16, compile-time Stockham plan (radix-16 stages, remainder last) and
// the LDS padding rule.  Included through fft_engine.h by every FFT kernel file.
#pragma once

#include <hip/hip_runtime.h>

namespace ocean {
namespace fftcore {

constexpr int kElems = 16;  // complex values held per lane per stage

constexpr int ilog2(int n) { return n <= 1 ? 0 : 1 + ilog2(n / 2); }
// Stockham plan: first stage radix R0 (16, 8 or 4), then radix-16 stages, the
// remainder (2/4/8/16) last.  R0 = 16 is the plain plan; the fused row pass
// uses R0 = 16 / planes so one lane holds every plane of its texels in stage 0.
constexpr int n_stages(int N, int R0 = 16) { return N <= R0 ? 1 : 1 + (ilog2(N) - ilog2(R0) + 3) / 4; }
constexpr int radix_of(int N, int s, int R0 = 16) {
    return s == 0 ? (N <= R0 ? N : R0)
                  : (s < n_stages(N, R0) - 1 ? 16 : (1 << (ilog2(N) - ilog2(R0) - 4 * (n_stages(N, R0) - 2))));
}
constexpr int ns_of(int N, int s, int R0 = 16) { return s == 0 ? 1 : ns_of(N, s - 1, R0) * radix_of(N, s - 1, R0); }
__device__ __forceinline__ int pad(int i) { return i + (i >> 4); }
constexpr int padded(int n) { return n + (n >> 4); }

// column-tile width (columns per workgroup) and row count per workgroup
constexpr int col_tile(int N) { return (8192 / N) < 4 ? 4 : ((8192 / N) > N ? N : 8192 / N); }
// width of the fused path's tile-major intermediate and foam state: the column
// tile for N <= 1024; 16 (128-byte rows) for the four-step column passes above
constexpr int inter_w(int N) { return N >= 2048 ? 16 : col_tile(N); }
// column-tile width of pass B (N <= 1024; the N >= 2048 column passes are four-step)
constexpr int b3_w(int N) { return N >= 2048 ? col_tile(N) : inter_w(N); }

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
// Complex multiply with fused multiply-adds (the FFT is not bound to the
// reference's rounding sequence: its parity is a norm-relative tolerance, and
// FMA is the more accurate form; the evolve / wave-data code that IS bit-exact
// lives in spectrum_math.h and is built without contraction).
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(fmaf(a.x, b.x, -(a.y * b.y)), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cmul_i(float2 a) { return make_float2(-a.y, a.x); }  // i * a

// exp(+2 pi i m / 16) for a compile-time m (0..15)
__device__ __forceinline__ float2 w16(int m) {
    constexpr float c1 = 0.923879532511286756f, s1 = 0.382683432365089772f, h = 0.707106781186547524f;
    const float cs[4] = {1.0f, c1, h, s1};
    const int q = (m >> 2) & 3, r = m & 3;
    float c = r == 0 ? 1.0f : cs[r], s = r == 0 ? 0.0f : cs[4 - r];
    // rotate by q quarter turns
    for (int k = 0; k < q; ++k) { float t = c; c = -s; s = t; }
    return make_float2(c, s);
}

// multiply by exp(+2 pi i m / 16), m compile-time after unrolling
__device__ __forceinline__ float2 rot16(float2 a, int m) {
    m &= 15;
    if (m == 0) return a;
    if (m == 4) return cmul_i(a);
    if (m == 8) return make_float2(-a.x, -a.y);
    if (m == 12) return make_float2(a.y, -a.x);
    return cmul(a, w16(m));
}

// In-register inverse DFT of radix R (sign +), R in {2, 4, 8, 16}.
template <int R>
struct Idft;
template <>
struct Idft<2> {
    static __device__ __forceinline__ void run(float2* v) {
        float2 a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    }
};
template <>
struct Idft<4> {
    static __device__ __forceinline__ void run(float2* v) {
        float2 a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
        float2 a2 = cadd(v[1], v[3]), a3 = cmul_i(csub(v[1], v[3]));
        v[0] = cadd(a0, a2);
        v[2] = csub(a0, a2);
        v[1] = cadd(a1, a3);
        v[3] = csub(a1, a3);
    }
};
// R = R1 * R2 with r = r1 + R1 r2, q = q2 + R2 q1:
// V[q] = sum_r1 w_R^(r1 q2) w_R1^(r1 q1) sum_r2 v[r1 + R1 r2] w_R2^(r2 q2)
template <int R>
struct Idft {
    static constexpr int R1 = (R == 8) ? 2 : 4;
    static constexpr int R2 = R / R1;
    static __device__ __forceinline__ void run(float2* v) {
        float2 t[R1][R2];
#pragma unroll
        for (int r1 = 0; r1 < R1; ++r1) {
#pragma unroll
            for (int r2 = 0; r2 < R2; ++r2) t[r1][r2] = v[r1 + R1 * r2];
            Idft<R2>::run(t[r1]);
#pragma unroll
            for (int q2 = 0; q2 < R2; ++q2) t[r1][q2] = rot16(t[r1][q2], r1 * q2 * (16 / R));
        }
#pragma unroll
        for (int q2 = 0; q2 < R2; ++q2) {
            float2 u[R1];
#pragma unroll
            for (int r1 = 0; r1 < R1; ++r1) u[r1] = t[r1][q2];
            Idft<R1>::run(u);
#pragma unroll
            for (int q1 = 0; q1 < R1; ++q1) v[q2 + R2 * q1] = u[q1];
        }
    }
};

// Twiddle + butterfly for one radix-R Stockham butterfly j at stage (NS, R).
template <int N, int R, int NS>
__device__ __forceinline__ void butterfly(float2* v, int j, const float2* __restrict__ tw) {
    if constexpr (NS > 1) {
        const int k = j & (NS - 1);
        constexpr int step = N / (NS * R);
#pragma unroll
        for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw[r * k * step]);
    }
    Idft<R>::run(v);
}

}  // namespace fftcore
}  // namespace ocean
