// The fused frame through a THREE-plane intermediate (N = 512 / 1024, full outputs):
// pass AQ (mirror-pair rows) and pass BQ (column tiles).  DESIGN.md section 3, "Three-plane frame".
//
// The reference transforms four packed planes (TimeDependentSpectrum.compute:42-45):
//   P1 = Dx + i Dz,  P2 = Dy + i Dxz,  P3 = Dyx + i Dyz,  P4 = Dxx + i Dzz
// and keeps the real / imaginary parts of each 2D IFFT T[.] (ResultTexturesFiller.compute:20-26).
// Re T[P] = T[herm P] and Im T[P] = T[anti P] / i, with herm P(k) = (P(k) + conj P(-k)) / 2 and
// anti P(k) = (P(k) - conj P(-k)) / 2 (-k = the mirror texel, InitialSpectrum.compute:139).
// Three of the four transforms the fill needs are therefore transforms of planes pass A can form
// per texel pair (k, -k), and the fourth differs from i kz P1 only on the two Nyquist lines:
//   Q1 = P1                         T[Q1]  = Dx  + i Dz
//   Q2 = herm P2 + i herm P3        T[Q2]  = Dy  + i Dyx
//   Q3 = -i anti P3 + i herm P4     T[Q3]  = Dyz + i Dxx
//   Q4 = -i anti P2 + anti P4       T[Q4]  = Dxz + i Dzz
// Off the lines nx = 0 and nz = 0, Q4 = i kz Q1 exactly in real arithmetic (Dxz = i kz Dx and
// Dzz = i kz Dz texel by texel), and kz is constant along a row, so after the row transform R:
//   R[Q4](x, y) = i kz(y) R[Q1](x, y) + d0(y)        (y != 0; d0(y) = Q4 - i kz Q1 at texel nx = 0)
//   R[Q4](x, 0) = srow(x) = R[Q4 of row 0](x)        (row nz = 0 transformed by pass A)
// The planes Q1..Q3 (24 B / texel instead of 32) plus the per-unit side arrays d0 and srow are the
// whole intermediate; pass B forms R[Q4] from R[Q1] on load.  The outputs equal the four-plane
// frame's in real arithmetic, Nyquist lines included; in fp32 they differ by rounding only.
#include "fft_engine.h"
#include "spectrum_math.h"

namespace ocean {
namespace {

// (a + conj b) / 2 and (a - conj b) / 2
__device__ __forceinline__ float2 hsum(float2 a, float2 b) { return make_float2((a.x + b.x) * 0.5f, (a.y - b.y) * 0.5f); }
__device__ __forceinline__ float2 hdif(float2 a, float2 b) { return make_float2((a.x - b.x) * 0.5f, (a.y + b.y) * 0.5f); }

struct QTex {
    float2 q[3];
};

// Q1..Q3 at k (a) and at -k (b) from the reference planes P(k) = o, P(-k) = om.
__device__ __forceinline__ void q_planes(const Planes4& o, const Planes4& om, QTex& a, QTex& b) {
    const float2 h2 = hsum(o.p[1], om.p[1]), h3 = hsum(o.p[2], om.p[2]);
    const float2 a3 = hdif(o.p[2], om.p[2]), h4 = hsum(o.p[3], om.p[3]);
    a.q[0] = o.p[0];
    b.q[0] = om.p[0];
    a.q[1] = make_float2(h2.x - h3.y, h2.y + h3.x);  // h2 + i h3
    b.q[1] = make_float2(h2.x + h3.y, h3.x - h2.y);  // conj h2 + i conj h3
    a.q[2] = make_float2(a3.y - h4.y, h4.x - a3.x);  // i (h4 - a3)
    b.q[2] = make_float2(a3.y + h4.y, a3.x + h4.x);  // i conj (a3 + h4)
}

// Q1..Q3 at k and -k straight from h = h(k, t) and the texel's wave data w = (kx, 1/|k|, kz, .),
// for a texel pair off the Nyquist lines (there h(-k) = conj h, and the mirror's wave data is
// (-kx, 1/|k|, -kz)): with P1..P4 of TimeDependentSpectrum.compute:29-45,
//   Q1 = P1 = (i kx - kz) / |k| h,  Q2 = Y + i Dyx = (1 - kx) h,  Q3 = Dyz + i Dxx = i (kz - kx^2 / |k|) h,
// and at -k the same with kx, kz negated and conj h: a complex scale of h each, 24 VALU for the pair
// where planes_of twice + q_planes take ~80 (pass A is VALU-heavy: SQ counters, docs/MEASUREMENTS.md section 6).  The
// same values in real arithmetic; in fp32 they round differently (parity tolerance, tests).
__device__ __forceinline__ void q_fast(float2 h, float4 w, QTex& a, QTex& b) {
    const float c1x = -w.z * w.y, c1y = w.x * w.y;  // (i kx - kz) / |k|
    a.q[0] = make_float2(c1x * h.x - c1y * h.y, c1x * h.y + c1y * h.x);
    b.q[0] = make_float2(-(c1x * h.x + c1y * h.y), c1x * h.y - c1y * h.x);  // -(c1) conj h
    const float s2a = 1.0f - w.x, s2b = 1.0f + w.x;
    a.q[1] = make_float2(s2a * h.x, s2a * h.y);
    b.q[1] = make_float2(s2b * h.x, -s2b * h.y);
    const float kk = w.x * w.x * w.y;
    const float t1 = w.z - kk, t2 = -w.z - kk;
    a.q[2] = make_float2(-t1 * h.y, t1 * h.x);  // i t1 h
    b.q[2] = make_float2(t2 * h.y, t2 * h.x);   // i t2 conj h
}

// Q4(k) - i kz(k) P1(k), nonzero only on the Nyquist lines (see the header).
__device__ __forceinline__ float2 q4_minus(const Planes4& o, const Planes4& om, float kz) {
    const float2 a2 = hdif(o.p[1], om.p[1]), a4 = hdif(o.p[3], om.p[3]);
    // -i a2 + a4 - i kz p1
    return make_float2(a2.y + a4.x + kz * o.p[0].y, -a2.x + a4.y - kz * o.p[0].x);
}
// Q4(k) itself (row nz = 0, whose transform is srow)
__device__ __forceinline__ float2 q4_full(const Planes4& o, const Planes4& om) {
    const float2 a2 = hdif(o.p[1], om.p[1]), a4 = hdif(o.p[3], om.p[3]);
    return make_float2(a2.y + a4.x, -a2.x + a4.y);
}

// The per-texel factors of texel x of row y that its row mirror N - x shares (nx negated, the same
// |k|): the phase factor e = exp(i omega t) and 1/|k| as (e.x, e.y, 1/|k|, 0); (1, 0, 1, 0) outside
// the cascade's band (wave_data's (kx, 1, kz, 0)).  omega = sqrt(g |k|) is correctly rounded as in
// wave_data (the phase omega t of a large t depends on its last bit); 1/|k| is the hardware
// reciprocal (1 ulp, inside the fp32 tolerance the three-plane passes are held to).
template <int N>
__device__ __forceinline__ float4 mirror_factors(int x, int y, const WaveBand& wb, float g, float time) {
    const float kx = (float)(x - N / 2) * wb.dk, kz = (float)(y - N / 2) * wb.dk;
    const float kmag = sqrtf(kx * kx + kz * kz);
    if (!(kmag >= wb.lo && kmag <= wb.hi)) return make_float4(1.0f, 0.0f, 1.0f, 0.0f);
    const Phase e = evolve_phase(sqrtf(g * kmag), time);
    return make_float4(e.ex, e.ey, __builtin_amdgcn_rcpf(kmag), 0.0f);
}

// Side arrays of unit u (of the chunk the view covers): d0 [N], then srow [N].
__device__ __forceinline__ float2* q_side(const DevView& v, int u) { return v.qside + (size_t)u * 2 * v.n; }

// Pass AQ: mirror-pair row pass writing Q1..Q3 (the structure of k_pass_a4, fft3.hip).  Item i
// of a unit (0 <= i <= N/2) is row y1 = i with its mirror row y2 = (N - i) % N; items 0 and N/2
// are self-mirror rows (y2 = y1), run by the same code: their second sequences duplicate the
// first and are not stored, except that item 0 carries srow in its second Q3 slot.  Lane j
// evolves texels x = j + r N/4 of row y1 with their mirrors (N - x) % N in row y2 and holds
// stage-0 butterfly j of row y1 and jm = (N/4 - j) % (N/4) of row y2.  LDS pass 0: Q1, Q2 of both
// rows; pass 1: Q3 of both rows in slots 2, 3 (slots 0, 1 idle, their butterflies skipped).
// OFF32: the intermediate stores take a scalar unit base and a 32-bit lane offset (plane, row, tile,
// column) instead of a 64-bit address (cfg3 pass A 29.15-29.40 -> 28.26-29.15 us); the host checks
// that the chunk's three planes lie within 4 GiB of the base (go_aq), else the 64-bit form runs.
// Three workgroups per CU (43.5 KiB of LDS each at N = 1024) need <= 168 VGPRs: the split pass 1 below
// takes 170 unconstrained, 168 with two spilled.
template <int N, bool BAND = false, int WT = 0, bool OFF32 = true>
__global__ __launch_bounds__(N / 4) __attribute__((amdgpu_waves_per_eu(N == 1024 ? 3 : 1, N == 1024 ? 3 : 10))) void
k_pass_aq(DevView v, float time, int items) {
    constexpr int R0 = 4, NJ = N / R0;
    constexpr int IPU = N / 2 + 1;  // items per unit
    using TW = StageTw<N, R0>;
    using E = Engine<N, 4, false, true, R0, TW, kElems>;
    constexpr int T = E::THREADS;
    static_assert(T == NJ && E::R0 == R0, "lane j <-> stage-0 butterfly j");
    constexpr int W = WT ? WT : inter_w(N);
    constexpr int TILES = N / W;
    constexpr int NSL = N / E::RL;
    static_assert(NSL % W == 0, "tile-major emit");
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    TW::load(twl, v.tw, threadIdx.x, T);
    const float2* tws = TW::table(twl, v.tw);
    __shared__ WaveBand band[kMaxCascades];
    if ((int)threadIdx.x < v.C) band[threadIdx.x] = wave_band(v.casc + threadIdx.x * 5);
    const int j = (int)threadIdx.x;
    const int jm = (NJ - j) & (NJ - 1);
    const bool j0 = (j == 0);
    auto rows_of = [&](int it, int& u, int& y1, int& y2) {
        u = it / IPU;
        y1 = it - u * IPU;
        y2 = (N - y1) & (N - 1);
    };
    auto load_pair = [&](int it, float2 (&a)[R0], float2 (&b)[R0]) {
        int u, y1, y2;
        rows_of(it, u, y1, y2);
        const float2* r1 = v.h0k + ((size_t)u * N + y1) * N;
        const float2* r2 = v.h0k + ((size_t)u * N + y2) * N;
#pragma unroll
        for (int r = 0; r < R0; ++r) {
            a[r] = r1[j + r * NJ];
            b[r] = r2[(N - j - r * NJ) & (N - 1)];
        }
    };
    auto unmirror = [&](const float2* mir, float2* out) {
#pragma unroll
        for (int r2 = 0; r2 < R0; ++r2) out[r2] = j0 ? mir[(R0 - r2) & (R0 - 1)] : mir[R0 - 1 - r2];
    };
    auto put = [&](int b, int jb, const float2* x) {
        float2* dst = lds + E::lidx(b, jb * R0);
#pragma unroll
        for (int q = 0; q < R0; ++q) dst[E::loff(q, 1)] = x[q];
    };
    float2 A[R0], B[R0], An[R0], Bn[R0];
    int it = blockIdx.x;
    if (it < items) load_pair(it, A, B);
    __syncthreads();  // twiddles, band
    for (; it < items; it += gridDim.x) {
        const int next = it + gridDim.x;
        if (next < items) load_pair(next, An, Bn);
        int u, y1, y2;
        rows_of(it, u, y1, y2);
        const WaveBand wb = band[(u + v.c0) % v.C];
        const bool self = (y1 == y2);
        const Win wunit = make_win(v.tplane + (size_t)u * TILES * N * W, 0);
        // after stage 0: g = (Q1 y1, Q1 y2, Q2 y1, Q2 y2, Q3 y1, Q3 y2 | row 0: srow's input)
        float2 g[6][R0];
        {
            float2 mir[3][R0];
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                // hardware reciprocal for 1/|k| (mirror_factors); omega and the phase as wave_data's
                const float4 f = mirror_factors<N>(j + r * NJ, y1, wb, v.gravity, time);
                const float4 wd = make_float4((float)(j + r * NJ - N / 2) * wb.dk, f.z, (float)(y1 - N / 2) * wb.dk, 0.0f);
                const float2 h = evolve_h(make_float4(A[r].x, A[r].y, B[r].x, -B[r].y), Phase{f.x, f.y});
                QTex qa, qb;
                if (y1 != 0 && !(r == 0 && j0)) {
                    q_fast(h, wd, qa, qb);
                } else {
                    // Nyquist lines: the mirror keeps kx on the column x = 0 and kz on the row y = 0
                    const float4 wm = make_float4((j0 && r == 0) ? wd.x : -wd.x, wd.y, y1 ? -wd.z : wd.z, wd.w);
                    const Planes4 o = planes_of(h, wd), om = planes_of(make_float2(h.x, -h.y), wm);
                    q_planes(o, om, qa, qb);
                    if (y1 == 0) qb.q[2] = q4_full(o, om);  // row 0: srow's input in the second Q3 slot
                    if (r == 0 && j0) {  // texel nx = 0 of both rows: d0
                        float2* side = q_side(v, u);
                        side[y1] = q4_minus(o, om, wd.z);
                        side[y2] = q4_minus(om, o, wm.z);
                    }
                }
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    g[2 * p][r] = qa.q[p];
                    mir[p][r] = qb.q[p];
                }
            }
            unmirror(mir[0], g[1]);
            unmirror(mir[1], g[3]);
            unmirror(mir[2], g[5]);
            if (y1 == 0) {  // srow's input stays in natural order (butterfly j)
#pragma unroll
                for (int r = 0; r < R0; ++r) g[5][r] = mir[2][r];
            }
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) Idft<R0>::run(g[k]);
        // SPLIT (N = 1024, wave-private stages): pass 1 (Q3 of both rows) runs on waves 2, 3 (slots 2, 3),
        // and the barrier that closes it is the next item's first one, so waves 0, 1 evolve the next item
        // meanwhile (cfg3 pass A 28.5-29.0 -> 27.4-28.0 us).  At N = 512 (two waves, stages with barriers)
        // pass 1 stays in slots 0, 1 behind a closing barrier: the split form there is 1.8 % slower
        // (docs/MEASUREMENTS.md section 8).
        constexpr bool SPLIT = E::wave_private(1);
        constexpr int Q3SLOT = SPLIT ? 2 : 0;
#pragma unroll
        for (int ps = 0; ps < 2; ++ps) {
            if (ps == 0) {
                if (SPLIT) __syncthreads();  // the previous item's pass 1 (waves 2, 3) has read slots 2, 3
#pragma unroll
                for (int k = 0; k < 4; ++k) put(k, (k & 1) ? jm : j, g[k]);
            } else {
                put(Q3SLOT, j, g[4]);
                put(Q3SLOT + 1, y1 ? jm : j, g[5]);
            }
            __syncthreads();
            auto emit = [&](int m, int q, float2 val) {
                int b, jj;
                E::template bj<E::RL>((int)threadIdx.x + m * T, b, jj);
                const int p = ps == 0 ? (b >> 1) : 2;
                const int s = b & 1;
                if (ps == 1 && (b >> 1) != (Q3SLOT >> 1)) return;  // idle slots
                const int x = jj + q * NSL;
                if (s && self) {  // self-mirror row: a duplicate, or row 0's srow
                    if (p == 2 && y1 == 0) q_side(v, u)[N + x] = val;
                    return;
                }
                if (BAND && (unsigned)(x - v.x0) >= (unsigned)v.nx) return;  // outside the column band
                if constexpr (OFF32) {
                    // scalar unit base + a 32-bit lane offset (plane, row, tile, column; < 4 GiB, go_aq):
                    // one 32-bit add per store instead of a 64-bit address
                    const unsigned off = (unsigned)p * (unsigned)(v.inter_stride * 8) +
                                         (unsigned)((((s ? y2 : y1) * W) + (jj / W) * N * W + (jj % W)) * 8);
                    *(float2*)(wunit.p + (store_off_t)(off + (unsigned)(q * (NSL / W) * N * W * 8))) = val;
                } else {
                    float2* dst = v.tplane + (size_t)p * v.inter_stride +
                                  ((size_t)u * TILES * N + (s ? y2 : y1)) * W + (size_t)(jj / W) * N * W + (jj % W);
                    dst[(size_t)q * (NSL / W) * N * W] = val;
                }
            };
            // pass 1: two sequence slots idle, their butterflies skipped (at N = 1024 the stages are
            // wave-private, wave w = sequence w: waves 0, 1 skip them whole and go on to the next item)
            E::template stages_from<1>(lds, tws, emit, ps == 1 ? Q3SLOT + 2 : 4, ps == 1 ? Q3SLOT : 0);
            if (ps == 0 || !SPLIT) __syncthreads();
        }
#pragma unroll
        for (int r = 0; r < R0; ++r) {
            A[r] = An[r];
            B[r] = Bn[r];
        }
    }
}

// Pass A3Q (N = 4096): the three-plane row pass in the shape of k_pass_a3 (fft3.hip):
// one row per item, lane j holds texels j + r N/4 (r < 4) of the sequences Q1, Q2, Q3 and, on row 0,
// srow's input (Q4 of row 0).  P(-k) is formed from the lane's own texel: h(-k) = conj h(k) bit for
// bit (h0.zw = conj h0(-k) after ocean_init_spectrum), with the mirror's wave data (kx, kz negated
// except on the Nyquist column / row).  16-wide tile-major intermediate as pass A3.  The LDS stages
// skip the idle fourth sequence slot (its butterflies' lanes only join the stage barriers); row 0 runs
// srow's input through them in a second pass (one row in N).  The next row's h0 is loaded right after
// the evolve has read the current row's, in flight across the row's stages (567 -> 517 us at cfg5).
template <int N, bool BAND = false>
__global__ __launch_bounds__(N / 4) void k_pass_a3q(DevView v, float time, int total_rows) {
    constexpr int FIRST = 4;
    using TW = StageTwLds<N, FIRST>;
    using E = Engine<N, 4, false, true, FIRST, TW>;
    constexpr int T = E::THREADS;
    constexpr int R0 = E::R0;
    constexpr int NJ = N / R0;
    constexpr int W = inter_w(N);
    constexpr int TILES = N / W;
    constexpr int NSL = N / E::RL;
    static_assert(T == NJ && R0 == 4, "lane j <-> stage-0 butterfly j of each sequence");
    __shared__ __align__(16) float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    TW::load(twl, v.tw, threadIdx.x, T);
    const float2* tws = TW::table(twl, v.tw);
    __shared__ WaveBand band[kMaxCascades];
    if ((int)threadIdx.x < v.C) band[threadIdx.x] = wave_band(v.casc + threadIdx.x * 5);
    const int j = (int)threadIdx.x;
    const bool j0 = (j == 0);
    float4 h[R0];
    auto load = [&](int item, float4* hh) {
        const Win w = make_win(v.h0 + (size_t)item * N, (unsigned)(N * 16));
#pragma unroll
        for (int r = 0; r < R0; ++r) hh[r] = bload4(w, j * 16, r * NJ * 16);
    };
    // deal consecutive rows to one XCD (blockIdx b runs on XCD b % 8), as pass A3
    int item = (gridDim.x % 8 == 0) ? (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)blockIdx.x / 8
                                    : (int)blockIdx.x;
    if (item < total_rows) load(item, h);
    __syncthreads();  // twiddles, band
    for (; item < total_rows; item += gridDim.x) {
        const int u = item / N, y = item % N;
        const WaveBand wb = band[(u + v.c0) % v.C];
        float2 in[4 * R0];  // slot p * R0 + r: sequence p, stage-0 input r
#pragma unroll
        for (int r = 0; r < R0; ++r) {
            const float4 wd = wave_data(j + r * NJ, y, N, wb, v.gravity);
            const float2 hh = evolve_h(h[r], evolve_phase(wd.w, time));
            QTex qa, qb;
            in[3 * R0 + r] = make_float2(0.0f, 0.0f);
            if (y != 0 && !(r == 0 && j0)) {
                q_fast(hh, wd, qa, qb);
            } else {  // Nyquist lines (see pass AQ)
                const float4 wm = make_float4((j0 && r == 0) ? wd.x : -wd.x, wd.y, y ? -wd.z : wd.z, wd.w);
                const Planes4 o = planes_of(hh, wd), om = planes_of(make_float2(hh.x, -hh.y), wm);
                q_planes(o, om, qa, qb);
                if (y == 0) in[3 * R0 + r] = q4_full(o, om);
                if (r == 0 && j0) q_side(v, u)[y] = q4_minus(o, om, wd.z);
            }
#pragma unroll
            for (int p = 0; p < 3; ++p) in[p * R0 + r] = qa.q[p];
        }
        const int next = item + gridDim.x;
        if (next < total_rows) load(next, h);  // the next row's h0 in flight across this row's stages
        auto put = [&](int b, int jj, int q, float2 val) {
            const int x = jj + q * NSL;
            if (b == 3) {
                if (y == 0) q_side(v, u)[N + x] = val;  // srow
                return;
            }
            if (BAND && (unsigned)(x - v.x0) >= (unsigned)v.nx) return;  // outside the column band
            float2* rowp = v.tplane + (size_t)b * v.inter_stride + ((size_t)u * TILES * N + y) * W;
            float2* dst = rowp + (size_t)(jj / W) * N * W + (jj % W);
            dst[(size_t)q * (NSL / W) * N * W] = val;
        };
#pragma unroll
        for (int p = 0; p < 4; ++p) Idft<R0>::run(&in[p * R0]);
        // pass 0: Q1..Q3 (sequence slot 3 idle); row 0 only, pass 1: srow's input in slot 0
        for (int ps = 0; ps < (y == 0 ? 2 : 1); ++ps) {
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                if (ps && p) continue;
                float2* dst = lds + E::lidx(p, j * R0);
#pragma unroll
                for (int q = 0; q < R0; ++q) dst[E::loff(q, 1)] = in[(ps ? 3 : p) * R0 + q];
            }
            __syncthreads();
            auto emit = [&](int m, int q, float2 val) {
                int b, jj;
                E::template bj<E::RL>((int)threadIdx.x + m * T, b, jj);
                put(ps ? 3 : b, jj, q, val);
            };
            E::template stages_from<1>(lds, tws, emit, ps ? 1 : 3);
            if (y == 0) __syncthreads();  // LDS reused by pass 1
        }
        __syncthreads();
    }
}

// Pass A3PP (N = 4096, column parity b = v.xpar, ocean_set_column_parity): the row pass of a rank that
// owns the columns x = 2m + b.  With X[x] = sum_n a[n] e^{2 pi i n x / N} and n = n' + (N/2) h,
//   X[2m + b] = sum_{n' < N/2} z_b[n'] e^{2 pi i n' m / (N/2)},  z_b[n'] = (a[n'] + (-1)^b a[n' + N/2]) w_N^{b n'}
// (decimation in frequency), so the rank evolves the whole row (its h0k is read whole either way), forms
// z_b of each sequence with one radix-2 butterfly in registers and runs an N/2-point transform instead
// of the N-point one.  Rows are paired as pass AQ pairs them: item i of a unit is row y1 = i with
// y2 = (N - i) % N; lane j (N/4 lanes) loads h0k of texels x_r = j + r N/4 (r < 4) of row y1 and of
// their mirrors N - x_r in row y2 (h(-k) = conj h(k) from the pair), evaluates the per-texel factors
// once per texel pair and, through an LDS exchange, once per four texels (x and N - x of row y1 have the
// same |k|: 1/|k| from the hardware reciprocal, omega correctly rounded), and folds z_b for both rows:
// row y1 at stage-0 butterfly j, row y2 at butterfly jm = (N/4 - j) % (N/4).  The 2048-point plan starts
// with a radix-2 stage (2, 16, 16, 4), so each LDS stage has one radix-16 butterfly per lane (16 waves
// per workgroup).  Seven sequence slots: 0-2 Q1..Q3 of row y1, 3-5 of row y2, 6 row 0's srow.  The
// self-mirror rows 0 and N/2 run the same code; their y2 slots duplicate y1 and are not stored.  Outputs
// m < N/2 go to intermediate column m (compact); d0 is per row (texel 0).  The next pair's h0k is in
// flight across the stages (0.094 against 0.098 ms loaded after them).  OFF32: 32-bit byte offsets from
// the intermediate's base (host-checked < 4 GiB), else 64-bit addresses.
template <int N, bool OFF32 = true>
__global__ __launch_bounds__(N / 4) void k_pass_a3pp(DevView v, float time, int items) {
    constexpr int H = N / 2;  // transform length
    constexpr int FIRST = 2;
    using TW = StageTwCompactSub<H, N, FIRST>;
    using E = Engine<H, 8, false, true, FIRST, TW, 8 * FIRST>;
    constexpr int T = E::THREADS;
    constexpr int R0 = E::R0;
    constexpr int NJ = H / R0;  // lanes = texel stride
    constexpr int W = inter_w(N);
    constexpr int TILES = N / W;
    constexpr int NSL = H / E::RL;
    constexpr int IPU = N / 2 + 1;  // items per unit
    static_assert(T == NJ && R0 == FIRST && T == N / 4, "lane j <-> stage-0 butterfly j of every slot");
    __shared__ __align__(16) float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    static_assert(R0 * NJ * 16 <= E::LDS_ELEMS * 8, "the factor exchange fits the idle image");
    float4* xch = reinterpret_cast<float4*>(lds);  // (e.x, e.y, 1/|k|) of texel j + r NJ of row y1, r < R0
    TW::load(twl, v.tw, threadIdx.x, T);
    const float2* tws = twl;
    __shared__ WaveBand band[kMaxCascades];
    if ((int)threadIdx.x < v.C) band[threadIdx.x] = wave_band(v.casc + threadIdx.x * 5);
    const int j = (int)threadIdx.x;
    const bool j0 = (j == 0);
    const int jm = (NJ - j) & (NJ - 1);
    const int par = v.xpar;
    const float sgn = par ? -1.0f : 1.0f;
    // w_N^{b n'} at n' = j + r NJ (row y1) and jm + r NJ (row y2): NJ = N/4 and w_N^{n + N/4} = i w_N^n, so
    // two values and a quarter turn
    const float2 zt1 = par ? v.tw[j] : make_float2(1.0f, 0.0f);
    const float2 zt2 = par ? v.tw[jm] : make_float2(1.0f, 0.0f);
    auto z1_at = [&](int r) { return (r && par) ? cmul_i(zt1) : zt1; };
    auto z2_at = [&](int r) {  // slot i2(r) = 1 - r off lane 0, r on lane 0
        const int i2 = j0 ? r : 1 - r;
        return (i2 && par) ? cmul_i(zt2) : zt2;
    };
    auto rows_of = [&](int it, int& u, int& y1, int& y2) {
        u = it / IPU;
        y1 = it - u * IPU;
        y2 = (N - y1) & (N - 1);
    };
    float2 A[2 * R0], B[2 * R0];
    auto load_pair = [&](int it) {
        int u, y1, y2;
        rows_of(it, u, y1, y2);
        const float2* r1 = v.h0k + ((size_t)u * N + y1) * N;
        const float2* r2 = v.h0k + ((size_t)u * N + y2) * N;
#pragma unroll
        for (int r = 0; r < 2 * R0; ++r) {
            A[r] = r1[j + r * NJ];
            B[r] = r2[(N - j - r * NJ) & (N - 1)];
        }
    };
    int it = blockIdx.x;
    if (it < items) load_pair(it);
    __syncthreads();  // twiddles, band
    for (; it < items; it += gridDim.x) {
        int u, y1, y2;
        rows_of(it, u, y1, y2);
        const WaveBand wb = band[(u + v.c0) % v.C];
        const bool self = (y1 == y2);
        float4 own[R0];
#pragma unroll
        for (int r = 0; r < R0; ++r) {
            own[r] = mirror_factors<N>(j + r * NJ, y1, wb, v.gravity, time);
            xch[r * NJ + j] = own[r];
        }
        __syncthreads();
        float2 in[7][R0];  // slots 0-2 row y1, 3-5 row y2, 6 srow (stage-0 input order)
#pragma unroll
        for (int r = 0; r < R0; ++r) {
            float2 qa[2][4], qb[2][3];  // texel pairs r (lo) and r + R0 (hi): Q1..Q3 (+ row 0's Q4) at k, Q1..Q3 at -k
#pragma unroll
            for (int hi = 0; hi < 2; ++hi) {
                const int rr = r + hi * R0;
                float4 f;
                if (hi == 0) {
                    f = own[r];
                } else {
                    const int rp = j0 ? 2 * R0 - rr : 2 * R0 - 1 - rr;  // the in-row mirror's r' (< R0, or R0 on lane 0)
                    f = (rp < R0) ? xch[(rp & (R0 - 1)) * NJ + jm] : mirror_factors<N>(j + rr * NJ, y1, wb, v.gravity, time);
                }
                const float4 wd = make_float4((float)(j + rr * NJ - N / 2) * wb.dk, f.z, (float)(y1 - N / 2) * wb.dk, 0.0f);
                const float2 h = evolve_h(make_float4(A[rr].x, A[rr].y, B[rr].x, -B[rr].y), Phase{f.x, f.y});
                QTex a, b;
                qa[hi][3] = make_float2(0.0f, 0.0f);
                if (y1 != 0 && !(rr == 0 && j0)) {
                    q_fast(h, wd, a, b);
                } else {  // Nyquist lines (see pass AQ)
                    const float4 wm = make_float4((j0 && rr == 0) ? wd.x : -wd.x, wd.y, y1 ? -wd.z : wd.z, wd.w);
                    const Planes4 o = planes_of(h, wd), om = planes_of(make_float2(h.x, -h.y), wm);
                    q_planes(o, om, a, b);
                    if (y1 == 0) qa[hi][3] = q4_full(o, om);
                    if (rr == 0 && j0) {
                        float2* side = q_side(v, u);
                        side[y1] = q4_minus(o, om, wd.z);
                        side[y2] = q4_minus(om, o, wm.z);
                    }
                }
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    qa[hi][p] = a.q[p];
                    qb[hi][p] = b.q[p];
                }
            }
            // row y1: z[j + r NJ] = Q(x_r) + s Q(x_{r+R0});  row y2 (slot i2(r)): Q(N - x_{r+R0}) + s Q(N - x_r),
            // except lane 0, r = 0 (texels 0 and N/2 map onto themselves): Q(N - x_0) + s Q(N - x_R0)
            const bool swap2 = j0 && r == 0;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                if (p == 3 && y1 != 0) {
                    in[6][r] = make_float2(0.0f, 0.0f);
                    continue;
                }
                const float2 z1 = make_float2(qa[0][p].x + sgn * qa[1][p].x, qa[0][p].y + sgn * qa[1][p].y);
                in[p == 3 ? 6 : p][r] = par ? cmul(z1, z1_at(r)) : z1;
                if (p < 3) {
                    const float2 a2 = swap2 ? qb[0][p] : qb[1][p], b2 = swap2 ? qb[1][p] : qb[0][p];
                    const float2 z2 = make_float2(a2.x + sgn * b2.x, a2.y + sgn * b2.y);
                    in[3 + p][R0 - 1 - r] = par ? cmul(z2, z2_at(r)) : z2;  // position i2(r) off lane 0
                }
            }
        }
        // lane 0: iteration r belongs at position (R0 - r) & (R0 - 1), not R0 - 1 - r: rotate positions by one
        if (j0) {
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const float2 t = in[3 + p][R0 - 1];
#pragma unroll
                for (int q = R0 - 1; q > 0; --q) in[3 + p][q] = in[3 + p][q - 1];
                in[3 + p][0] = t;
            }
        }
        const int next = it + gridDim.x;
        if (next < items) load_pair(next);  // the next pair's h0k in flight across the stages
#pragma unroll
        for (int sl = 0; sl < 7; ++sl) Idft<R0>::run(in[sl]);
        __syncthreads();  // every lane has read the exchange off the image
        const int live = (y1 == 0) ? 7 : 6;
#pragma unroll
        for (int sl = 0; sl < 7; ++sl) {
            if (sl == 6 && y1 != 0) continue;
            float2* dst = lds + E::lidx(sl, ((sl >= 3 && sl < 6) ? jm : j) * R0);
#pragma unroll
            for (int q = 0; q < R0; ++q) dst[E::loff(q, 1)] = in[sl][q];
        }
        __syncthreads();
        auto emit = [&](int m, int q, float2 val) {
            int b, jj;
            E::template bj<E::RL>((int)threadIdx.x + m * T, b, jj);
            const int mm = jj + q * NSL;  // compact column: x = 2 mm + parity
            if (b == 6) {
                if (y1 == 0) q_side(v, u)[N + mm] = val;  // srow
                return;
            }
            if (b >= 3 && self) return;  // the self-mirror row's duplicate
            const int p = b >= 3 ? b - 3 : b;
            const int y = b >= 3 ? y2 : y1;
            if constexpr (OFF32) {
                const unsigned e = (unsigned)p * (unsigned)v.inter_stride + ((unsigned)u * TILES * N + (unsigned)y) * W +
                                   (unsigned)(jj / W) * N * W + (unsigned)(jj % W) + (unsigned)q * (NSL / W) * N * W;
                *(float2*)((char*)v.tplane + (store_off_t)(e * 8u)) = val;
            } else {
                float2* dst = v.tplane + (size_t)p * v.inter_stride + ((size_t)u * TILES * N + y) * W +
                              (size_t)(jj / W) * N * W + (jj % W);
                dst[(size_t)q * (NSL / W) * N * W] = val;
            }
        };
        E::template stages_from<1>(lds, tws, emit, live);
        __syncthreads();
    }
}

// Pass BQ: per (unit, W-column tile), four column transforms from three planes:
//   step 0: R[Q2] -> (Dy, Dyx)          kept (LDS)
//   step 1: R[Q1] -> (Dx, Dz)           DISP = (Dx, Dy, Dz, 1); Dyx moves to registers; before the
//                                       transform R[Q4] = i kz R[Q1] + d0 (row 0: srow) is formed
//                                       from the same registers into the next ring slot
//   step 2: R[Q4] -> (Dxz, Dzz)         kept (LDS)
//   step 3: R[Q3] -> (Dyz, Dxx)         foam (Dxx, Dzz, Dxz), TURB, DERIV = (Dyx, Dyz, Dxx, Dzz)
// Three tile loads per item run through a three-slot register ring (two steps ahead), as in
// k_pass_b3; d0 is staged through LDS.  DC (DevView::disp_cached): DISP with default-policy stores.
template <int N, bool BAND = false, int WT = 0, bool DC = false>
__global__ __launch_bounds__((WT ? WT : b3_w(N)) * N / kElems) void k_pass_bq(DevView v, int items) {
    using CT = ColTile<N, WT ? WT : b3_w(N)>;
    using E = typename CT::E;
    using TW = typename CT::TW;
    constexpr int W = CT::W;
    constexpr int T = CT::T;
    constexpr int RL = CT::RL;
    constexpr int TILE = W * N;
    constexpr bool kKeepLds = (E::LDS_ELEMS + TW::kLdsEntries + kElems * T + N) * 8 <= 160 * 1024;
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    __shared__ float2 keep_lds[kKeepLds ? kElems * T : 1];
    __shared__ float dks[kMaxCascades];
    __shared__ float2 d0s[N];  // the item's d0, staged through LDS instead of 16 registers per lane
    constexpr int DPL = (N + T - 1) / T;  // d0 entries each lane stages
    TW::load(twl, v.tw, threadIdx.x, T);
    const float2* tws = TW::table(twl, v.tw);
    if ((int)threadIdx.x < v.C) dks[threadIdx.x] = wave_band(v.casc + threadIdx.x * 5).dk;
    const int lb = CT::lane_b(), lj = CT::lane_j();
    const int toff = lj * W + lb;
    const int voff16 = (lj * N + lb) * 16;

    float2 keep_reg[kKeepLds ? 1 : kElems];
    auto kput = [&](int i, float2 x) {
        if constexpr (kKeepLds) keep_lds[i * T + threadIdx.x] = x;
        else keep_reg[i] = x;
    };
    auto kget = [&](int i) -> float2 {
        if constexpr (kKeepLds) return keep_lds[i * T + threadIdx.x];
        else return keep_reg[i];
    };
    // item -> full tile index u * tiles + tile over the column band's tiles
    const int bt0 = v.x0 / W, bnt = v.nx / W;
    // Without DC (chunked frames, as cfg4's) the 32 workgroups of one XCD (blocks b, b + 8, ...) take 32
    // consecutive tiles at each step of the item loop, so each XCD streams whole 256-column runs of the
    // texture rows: cfg4 51.2 -> 52.0 k tile-frames/s (G = 64 the same, 128 slower); at cfg3 (DC) it does
    // not help (docs/MEASUREMENTS.md section 8).  Needs items % (8 G) == 0, else the identity order.
    constexpr int G = DC ? 1 : 32;
    const bool grp = G > 1 && items % (8 * G) == 0;
    auto full = [&](int item) {
        if (grp) item = (item & ~(8 * G - 1)) + G * (item & 7) + ((item >> 3) & (G - 1));
        return BAND ? (item / bnt) * CT::tiles + bt0 + item % bnt : item;
    };
    auto win16 = [&](const float4* base, int ft) {
        const int u = ft / CT::tiles, x0 = (ft % CT::tiles) * W;
        return make_win(base + (size_t)u * N * N + x0, (unsigned)((N * N - x0) * 16));
    };
    auto load = [&](int item, int p, float2 (&d)[kElems]) {
        const Win w = make_win(v.tplane + (size_t)p * v.inter_stride + (size_t)full(item) * TILE, TILE * 8);
        // DC: the intermediate's loads are nontemporal too (it is dead once read), which leaves DISP the
        // cache room; together +1.1-2.1 % at cfg3.  Without DC (chunked frames) they stay default-policy: at cfg4
        // nontemporal loads measured -1.1 to +1.1 % on two boxes (docs/MEASUREMENTS.md section 8)
#pragma unroll
        for (int i = 0; i < kElems; ++i)
            d[i] = DC ? bload2<2>(w, toff * 8, CT::in_dy(i) * W * 8) : bload2(w, toff * 8, CT::in_dy(i) * W * 8);
    };

    float2 cur[kElems], nxt[kElems], nx2[kElems], dd[DPL], srow = make_float2(0.0f, 0.0f);
    float kreg[kElems];
    int item = blockIdx.x;
    if (item < items) {
        load(item, 1, cur);  // R[Q2]
        load(item, 0, nxt);  // R[Q1]
    }
    __syncthreads();
    for (; item < items; item += gridDim.x) {
        const int ft = full(item);
        const int u = ft / CT::tiles;
        const int x0 = (ft % CT::tiles) * W;
        const float dk = dks[(u + v.c0) % v.C];
        float* foam = v.foam + (size_t)ft * TILE + toff;
        float fb[kElems];
        const bool more = item + (int)gridDim.x < items;
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            if (st == 0) {  // side values for step 1: the unit's d0 and, on row-0 lanes, srow
                const float2* side = q_side(v, u);
#pragma unroll
                for (int k = 0; k < DPL; ++k)
                    if (k * T + (int)threadIdx.x < N) dd[k] = side[k * T + threadIdx.x];
                if (lj == 0) srow = side[N + x0 + lb];
                load(item, 2, nx2);  // R[Q3]
            } else if (st == 1) {
                // R[Q4] = i kz R[Q1] + d0 (row 0: srow) into the free ring slot
#pragma unroll
                for (int r = 0; r < kElems; ++r) {
                    const int y = lj + CT::in_dy(r);
                    const float kz = (float)(y - N / 2) * dk;
                    const float2 c = cur[r], d = d0s[y];
                    nx2[r] = make_float2(d.x - kz * c.y, d.y + kz * c.x);
                }
                if (lj == 0) nx2[0] = srow;
            } else {
                if (st == 2) {  // foam state for step 3, ahead of this step's prefetch
                    const Win rf = make_win(v.foam + (size_t)ft * TILE, TILE * 4);
#pragma unroll
                    for (int m = 0; m < kElems / RL; ++m)
#pragma unroll
                        for (int q = 0; q < RL; ++q) fb[m * RL + q] = bload1(rf, toff * 4, CT::out_dy(m, q) * W * 4);
                }
                if (more) load(item + gridDim.x, st == 2 ? 1 : 0, nx2);  // next item's R[Q2], R[Q1]
            }
            const Win wd = win16(v.disp, ft), wt = win16(v.turb, ft), wv = win16(v.deriv, ft);
            auto emit = [&](int m, int q, float2 val) {
                const int i = m * RL + q;
                const int dy = CT::out_dy(m, q);
                const float s = perm_sign(x0 + lb, lj + dy);
                const float re = val.x * s, im = val.y * s;
                const int so = dy * N * 16;
                if (st == 0) {  // (Dy, Dyx)
                    kput(i, make_float2(re, im));
                } else if (st == 1) {  // (Dx, Dz): DISP
                    const float2 k = kget(i);
                    if constexpr (DC) gstore4(make_float4(re, k.x, im, 1.0f), wd, voff16, so);
                    else gstore4_nt(make_float4(re, k.x, im, 1.0f), wd, voff16, so);
                    kreg[i] = k.y;
                } else if (st == 2) {  // (Dxz, Dzz)
                    kput(i, make_float2(re, im));
                } else {  // (Dyz, Dxx): foam, TURB, DERIV, NORMAL
                    const float2 k = kget(i);  // (Dxz, Dzz)
                    const float f = foam_update(fb[i], im, k.y, k.x);
                    foam[dy * W] = f;
                    gstore4_nt(make_float4(f, f, f, f), wt, voff16, so);
                    gstore4_nt(make_float4(kreg[i], re, im, k.y), wv, voff16, so);
                    if (v.normals) gstore4_nt(normal_from_deriv(kreg[i], re, im, k.y), win16(v.normal, ft), voff16, so);
                }
            };
            E::run_regs(cur, lds, tws, emit);
            if (st == 0) {
#pragma unroll
                for (int k = 0; k < DPL; ++k)
                    if (k * T + (int)threadIdx.x < N) d0s[k * T + threadIdx.x] = dd[k];
            }
            // ring: after step 1 the formed R[Q4] (nx2) goes first and R[Q3] (nxt) stays next
#pragma unroll
            for (int i = 0; i < kElems; ++i) {
                if (st == 1) {
                    cur[i] = nx2[i];
                } else {
                    cur[i] = nxt[i];
                    nxt[i] = nx2[i];
                }
            }
            __syncthreads();
        }
    }
}

template <class K>
int grid_q(K kernel, int threads, int items) {
    const int g = device_cus() * resident_per_cu((const void*)kernel, threads);
    return items < g ? items : g;
}

// Byte offsets of a store into the chunk's intermediate planes 0..2 fit 32 bits (k_pass_aq /
// k_pass_a3pp OFF32): the last byte of plane 2 lies below 4 GiB from the base.
bool inter_off32(const DevView& v) { return ((size_t)2 * v.inter_stride + v.inter_stride) * 8 <= ((size_t)1 << 32); }

template <int N, bool BAND = false, int WT = 0, bool OFF32 = true>
hipError_t go_aq(const DevView& v, float t, hipStream_t s) {
    if constexpr (WT == 0) {
        if (v.tile_w != inter_w(N)) return go_aq<N, BAND, 4, OFF32>(v, t, s);
    }
    if constexpr (!BAND) {
        if (v.nx != N) return go_aq<N, true, WT, OFF32>(v, t, s);
    }
    if constexpr (OFF32) {
        if (!inter_off32(v)) return go_aq<N, BAND, WT, false>(v, t, s);
    }
    constexpr int T = N / 4;
    const int items = v.units * (N / 2 + 1);
    const int g = grid_q(k_pass_aq<N, BAND, WT, OFF32>, T, items);
    launch((k_pass_aq<N, BAND, WT, OFF32>), dim3(g), dim3(T), 0, s, v, t, items);
    return hipGetLastError();
}

template <int N, bool BAND = false>
hipError_t go_a3q(const DevView& v, float t, hipStream_t s) {
    if constexpr (!BAND) {
        if (v.nx != N) return go_a3q<N, true>(v, t, s);
    }
    constexpr int T = N / 4;
    const int total = v.units * N;
    const int g = grid_q(k_pass_a3q<N, BAND>, T, total);
    launch((k_pass_a3q<N, BAND>), dim3(g), dim3(T), 0, s, v, t, total);
    return hipGetLastError();
}

template <int N, bool BAND = false, int WT = 0, bool DC = false>
hipError_t go_bq(const DevView& v, hipStream_t s) {
    if constexpr (WT == 0) {
        if (v.tile_w != inter_w(N)) return go_bq<N, BAND, 4, DC>(v, s);
    }
    if constexpr (!BAND) {
        if (v.nx != N) return go_bq<N, true, WT, DC>(v, s);
    }
    if constexpr (!DC) {
        if (v.disp_cached) return go_bq<N, BAND, WT, true>(v, s);
    }
    constexpr int W = WT ? WT : b3_w(N);
    constexpr int T = W * N / kElems;
    const int items = v.units * (v.nx / W);
    const int g = grid_q(k_pass_bq<N, BAND, WT, DC>, T, items);
    launch((k_pass_bq<N, BAND, WT, DC>), dim3(g), dim3(T), 0, s, v, items);
    return hipGetLastError();
}

}  // namespace

// N = 2048 keeps the four-plane passes: pass A3Q's idle fourth sequence slot costs more there
// than the column passes save (4 x 2048^2: 612 against 599 us per frame; docs/MEASUREMENTS.md section 3).
bool pass_q_supported(int n, int planes) { return planes == 4 && (n == 512 || n == 1024 || n == 4096); }

hipError_t launch_pass_a_q(const DevView& v, float t, hipStream_t s) {
    if (!pass_q_supported(v.n, v.planes) || !v.qside) return hipErrorInvalidValue;
    if (v.xstr == 2) {  // column parity (even / odd columns of every row): pass A3PP on mirror-pair rows
        if (v.n != 4096 || v.x0 != 0 || v.nx != v.n / 2 || !v.h0k) return hipErrorInvalidValue;
        constexpr int T = 4096 / 4;
        const int items = v.units * (4096 / 2 + 1);
        if (inter_off32(v)) {
            const int g = grid_q(k_pass_a3pp<4096, true>, T, items);
            launch((k_pass_a3pp<4096, true>), dim3(g), dim3(T), 0, s, v, t, items);
        } else {
            const int g = grid_q(k_pass_a3pp<4096, false>, T, items);
            launch((k_pass_a3pp<4096, false>), dim3(g), dim3(T), 0, s, v, t, items);
        }
        return hipGetLastError();
    }
    switch (v.n) {
        case 512: return v.h0k ? go_aq<512>(v, t, s) : hipErrorInvalidValue;
        case 1024: return v.h0k ? go_aq<1024>(v, t, s) : hipErrorInvalidValue;
        case 4096: return go_a3q<4096>(v, t, s);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_pass_b_q(const DevView& v, hipStream_t s) {
    if (!pass_q_supported(v.n, v.planes) || v.n > 1024 || !v.qside) return hipErrorInvalidValue;
    return v.n == 512 ? go_bq<512>(v, s) : go_bq<1024>(v, s);
}

}  // namespace ocean
