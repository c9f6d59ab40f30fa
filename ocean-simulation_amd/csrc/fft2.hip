// The operator IFFT (ocean_ifft2d = IFFT.InverseFastFourierTransform,
// IFFT.cs:66-94) for gfx950: an in-place row launch and an in-place column +
// permute launch per run of planes.
//  * persistent grid (CUs x resident workgroups); each workgroup walks items
//    (rows / column tiles) with stride gridDim.x;
//  * the next item's global loads are issued into registers before the current
//    item's FFT stages and stores (vmcnt counts loads and stores in issue order,
//    so the prefetch goes out first);
//  * global loads use buffer_load with one 32-bit voffset per lane and the
//    per-element stride in the scalar soffset; stores are plain global stores
//    (fft_engine.h, memory ops);
//  * every LDS access of a butterfly is (per-lane base) + (compile-time
//    offset), twiddles come from per-stage LDS tables (fft_engine.h).
#include <cstdlib>

#include "fft_engine.h"

namespace ocean {
namespace {

// -------------------------------------------------------------- kernels
// rows per workgroup of k_rows2: 4 at N = 1024 (1024 lanes); one row (256 lanes, 3 workgroups per CU)
// at N = 2048 / 4096, where a 4-row image (128 / 256 KiB) held one workgroup per CU
constexpr int rows_per_item(int N) { return N >= 2048 ? 1 : (N >= 1024 ? 4 : 4096 / N); }

// Standalone row pass, in place: item = B consecutive rows of the flattened
// [unit][y] row list of one plane.
// `dst` may equal `plane` (in place) or be a scratch buffer of the same layout (the N >= 2048
// four-step operator below).
template <int N, int B = rows_per_item(N)>
__global__ __launch_bounds__(B * N / kElems) void k_rows2(const float2* plane, float2* dst, int total_rows,
                                                         const float2* __restrict__ tw) {
    using TW = StageTwLds<N>;
    using E = Engine<N, B, false, true, 16, TW>;
    constexpr int T = E::THREADS;
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    TW::load(twl, tw, threadIdx.x, T);
    const float2* tws = TW::table(twl, tw);
    const int items = (total_rows + B - 1) / B;
    float2 cur[kElems], nxt[kElems];
    auto load = [&](int item, float2 (&d)[kElems]) {
        const int rows = min(B, total_rows - item * B);
        const Win w = make_win(plane + (size_t)item * B * N, (unsigned)(rows * N * 8));
#pragma unroll
        for (int m = 0; m < kElems / E::R0; ++m) {
            int b, j;
            E::template bj<E::R0>((int)threadIdx.x + m * T, b, j);
#pragma unroll
            for (int q = 0; q < E::R0; ++q) d[m * E::R0 + q] = bload2(w, (b * N + j) * 8, q * (N / E::R0) * 8);
        }
    };
    int item = blockIdx.x;
    if (item < items) load(item, cur);
    __syncthreads();  // twiddle table
    for (; item < items; item += gridDim.x) {
        const int next = item + gridDim.x;
        if (next < items) load(next, nxt);
        const Win w = make_win(dst + (size_t)item * B * N, 0);
        auto emit = [&](int m, int q, float2 val) {
            int b, j;
            E::template bj<E::RL>((int)threadIdx.x + m * T, b, j);
            if (item * B + b < total_rows) gstore2(val, w, (b * N + j) * 8, q * (N / E::RL) * 8);
        };
        E::run_regs(cur, lds, tws, emit);
#pragma unroll
        for (int i = 0; i < kElems; ++i) cur[i] = nxt[i];
        __syncthreads();
    }
}

// Standalone column pass + permute, in place: item = W columns of one unit.
// W = 16 at N = 1024 (128-byte row segments; 1024 lanes), col_tile(N) otherwise; at N = 1024 the
// default is W = 8 with XCD-paired halves (XP below): 2 workgroups per CU instead of 1, and every
// 128-byte line still moves through one L2.
constexpr int cols2_w(int N) { return N == 1024 ? 16 : col_tile(N); }

// G > 1 (XCD grouping): the G W-column pieces of a (G W)-column tile go to items i, i + 8, ...,
// i + 8 (G - 1), which blocks b, b + 8, ... -- one XCD under round-robin placement (speed only, never
// correctness) -- take at the same time, so each 128-byte line is fetched and written back through one
// L2.  G = 2, W = 8 at N = 1024; G = 4, W = 4 at N = 2048 / 4096 (OCEAN_COLS2_XQ).
template <int N, int W_ = cols2_w(N), int G = 1>
__global__ __launch_bounds__(W_ * N / kElems) void k_cols2(float2* __restrict__ plane, int items,
                                                          const float2* __restrict__ tw) {
    using CT = ColTile<N, W_>;
    using E = typename CT::E;
    using TW = typename CT::TW;
    constexpr int W = CT::W;
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    TW::load(twl, tw, threadIdx.x, CT::T);
    const float2* tws = TW::table(twl, tw);
    const int lb = CT::lane_b(), lj = CT::lane_j();
    const int voff = (lj * N + lb) * 8;
    float2 cur[kElems], nxt[kElems];
    // item -> tile index (unit * tiles + tile)
    auto tile_of = [&](int item) {
        if constexpr (G > 1) return (item & ~(8 * G - 1)) + G * (item & 7) + ((item >> 3) & (G - 1));
        else return item;
    };
    auto win = [&](int item) {
        const int t = tile_of(item);
        const int u = t / CT::tiles, x0 = (t - u * CT::tiles) * W;
        return make_win(plane + (size_t)u * N * N + x0, (unsigned)((N * N - x0) * 8));
    };
    auto load = [&](int item, float2 (&d)[kElems]) {
        const Win w = win(item);
#pragma unroll
        for (int i = 0; i < kElems; ++i) d[i] = bload2(w, voff, CT::in_dy(i) * N * 8);
    };
    int item = blockIdx.x;
    if (item < items) load(item, cur);
    __syncthreads();
    for (; item < items; item += gridDim.x) {
        const int next = item + gridDim.x;
        if (next < items) load(next, nxt);
        const Win w = win(item);
        const int x0 = (tile_of(item) % CT::tiles) * W;
        auto emit = [&](int m, int q, float2 val) {
            const int dy = CT::out_dy(m, q);
            const float s = perm_sign(x0 + lb, lj + dy);
            gstore2(make_float2(val.x * s, val.y * s), w, voff, dy * N * 8);
        };
        E::run_regs(cur, lds, tws, emit);
#pragma unroll
        for (int i = 0; i < kElems; ++i) cur[i] = nxt[i];
        __syncthreads();
    }
}

// ------------------------------------------------- four-step columns (N >= 2048)
// The column transform of the operator at N = 2048 / 4096 as two passes over standard-layout
// [y][x] unit-planes (the frame's fft4k.hip passes run on its tile-major intermediate instead):
// N = L1 * L0, L1 = 64, y = y1 + L1 y0, k = k0 + L0 k1,
//   C1 (in place): A[y1][k0] = w_N^(y1 k0) sum_y0 X[y1 + L1 y0] w_L0^(y0 k0), in the slot of X[y1 + L1 k0]
//   C2 (out of place): Y[k0 + L0 k1] = sum_y1 A[y1][k0] w_L1^(y1 k1), then the permute.
// A k_cols2 tile whose whole columns fit LDS at 4096 is 4 columns wide: 32-byte row pieces.  Here
// every access is a 128-byte row piece (16 columns).  C2's outputs (rows k0 + L0 k1) are other
// items' inputs (rows L1 k0 + y1), so the operator runs rows -> scratch, C1 on the scratch, C2
// scratch -> plane, per chunk of unit-planes small enough to stay in the Infinity Cache.
constexpr int kOpL1 = 64;                       // step-2 length
constexpr int kOpW = 16;                        // columns per tile: 128-byte row pieces
constexpr int kOpSeq = 64;                      // sequences per workgroup: 16 columns x 4 y1 (C1) / k0 (C2)
constexpr int kOpBlk = kOpSeq / kOpW;           // y1 (C1) or k0 (C2) values per item

// Per-stage tables of the L-point plan read from the context's N-point table tw[m] = exp(2 pi i m / N)
// (the same float bits as the frame's fft4k.hip SubTw).
template <int L, int N>
struct OpSubTw {
    using Full = StageTw<L, 16>;
    static constexpr int S = Full::S;
    static constexpr int kLdsEntries = Full::kEntries;
    template <int s>
    static __device__ __forceinline__ void load_stage(float2* lds, const float2* tw, int tid, int nthreads) {
        if constexpr (s < S) {
            constexpr int NS = ns_of(L, s, 16), R = radix_of(L, s, 16), O = Full::off(s);
            for (int i = tid; i < NS * R; i += nthreads) {
                const int r = i / NS, k = i % NS;
                lds[O + i] = tw[(r * k * (N / (NS * R))) & (N - 1)];
            }
            load_stage<s + 1>(lds, tw, tid, nthreads);
        }
    }
    static __device__ __forceinline__ void load(float2* lds, const float2* tw, int tid, int nthreads) {
        load_stage<1>(lds, tw, tid, nthreads);
    }
    template <int ST>
    static __device__ __forceinline__ void apply(float2* v, int j, const float2* tws) {
        Full::template apply<ST>(v, j, tws);
    }
};

// C1: item = (unit-plane, 16-column tile, block of 4 y1); sequence b = y1_local * 16 + column,
// element y0 at row y1 + L1 y0.  `buf` holds `ups` unit-planes of N x N.
template <int N>
__global__ __launch_bounds__(kOpSeq * (N / kOpL1) / kElems) void k_opc1(float2* __restrict__ buf, int items,
                                                                         const float2* __restrict__ tw) {
    constexpr int L0 = N / kOpL1;
    using CT = ColTile<L0, kOpSeq>;
    using TW = OpSubTw<L0, N>;
    using E = Engine<L0, kOpSeq, true, Engine<L0, kOpSeq, true, false>::seq_pad_ok(), 16, TW>;
    constexpr int T = E::THREADS;
    constexpr int TILES = N / kOpW;
    constexpr int BLKS = kOpL1 / kOpBlk;  // y1 blocks per tile
    constexpr int ES = kOpL1 * N;         // element (y0) stride in float2
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    __shared__ float2 two[128];  // w_N^m = lo[m % 64] * hi[m / 64]
    TW::load(twl, tw, threadIdx.x, T);
    for (int i = threadIdx.x; i < 128; i += T) two[i] = tw[N + i];
    const int lb = (int)threadIdx.x % kOpSeq, lj = (int)threadIdx.x / kOpSeq;
    const int col = lb % kOpW, y1l = lb / kOpW;
    const int voff = ((y1l + kOpL1 * lj) * N + col) * 8;  // lane's element from the item's base
    auto item_base = [&](int item) {  // uniform: unit-plane, tile, first y1 of the item
        const int blk = item % BLKS, ut = item / BLKS;
        const int up = ut / TILES, t = ut % TILES;
        return buf + (size_t)up * N * N + (size_t)blk * kOpBlk * N + t * kOpW;
    };
    auto base_of = [&](int item) { return item_base(item) + voff / 8; };
    float2 cur[kElems], nxt[kElems];
    auto load = [&](int item, float2 (&d)[kElems]) {
        const int blk = item % BLKS, t = (item / BLKS) % TILES;
        const Win w = make_win(item_base(item), (unsigned)((N * N - blk * kOpBlk * N - t * kOpW) * 8));
#pragma unroll
        for (int i = 0; i < kElems; ++i) d[i] = bload2(w, voff, CT::in_dy(i) * ES * 8);
    };
    int item = blockIdx.x;
    if (item < items) load(item, cur);
    __syncthreads();
    for (; item < items; item += gridDim.x) {
        const int next = item + gridDim.x;
        if (next < items) load(next, nxt);
        float2* dst = base_of(item);
        const int y1 = (item % BLKS) * kOpBlk + y1l;
        auto emit = [&](int m, int q, float2 val) {
            const int dy = CT::out_dy(m, q);  // k0 - lj
            const int mm = y1 * (lj + dy);    // < L1 * L0 = N
            const float2 w = cmul(two[mm & 63], two[64 + (mm >> 6)]);
            dst[(size_t)dy * ES] = cmul(val, w);
        };
        E::run_regs(cur, lds, twl, emit);
#pragma unroll
        for (int i = 0; i < kElems; ++i) cur[i] = nxt[i];
        __syncthreads();
    }
}

// C2: item = (unit-plane, 16-column tile, block of 4 k0); sequence b = k0_local * 16 + column,
// element y1 at row L1 k0 + y1 of `src`; output row k0 + L0 k1 of `dst`, permuted.
template <int N>
__global__ __launch_bounds__(kOpSeq * kOpL1 / kElems) void k_opc2(const float2* __restrict__ src,
                                                                 float2* __restrict__ dst, int items,
                                                                 const float2* __restrict__ tw) {
    constexpr int L0 = N / kOpL1;
    using CT = ColTile<kOpL1, kOpSeq>;
    using TW = OpSubTw<kOpL1, N>;
    using E = Engine<kOpL1, kOpSeq, true, Engine<kOpL1, kOpSeq, true, false>::seq_pad_ok(), 16, TW>;
    constexpr int T = E::THREADS;
    constexpr int TILES = N / kOpW;
    constexpr int BLKS = L0 / kOpBlk;  // k0 blocks per tile
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    TW::load(twl, tw, threadIdx.x, T);
    const int lb = (int)threadIdx.x % kOpSeq, lj = (int)threadIdx.x / kOpSeq;
    const int col = lb % kOpW, k0l = lb / kOpW;
    auto decode = [&](int item, int& up, int& x, int& k0) {
        const int blk = item % BLKS, ut = item / BLKS;
        up = ut / TILES;
        x = (ut % TILES) * kOpW + col;
        k0 = blk * kOpBlk + k0l;
    };
    float2 cur[kElems], nxt[kElems];
    const int voff = ((kOpL1 * k0l + lj) * N + col) * 8;  // lane's element from the item's base
    auto load = [&](int item, float2 (&d)[kElems]) {
        const int blk = item % BLKS, ut = item / BLKS;
        const int up = ut / TILES, t = ut % TILES;
        const size_t o = (size_t)kOpL1 * kOpBlk * blk * N + t * kOpW;  // uniform: first k0 row, tile
        const Win w = make_win(src + (size_t)up * N * N + o, (unsigned)(((size_t)N * N - o) * 8));
#pragma unroll
        for (int i = 0; i < kElems; ++i) d[i] = bload2(w, voff, CT::in_dy(i) * N * 8);
    };
    int item = blockIdx.x;
    if (item < items) load(item, cur);
    __syncthreads();
    for (; item < items; item += gridDim.x) {
        const int next = item + gridDim.x;
        if (next < items) load(next, nxt);
        int up, x, k0;
        decode(item, up, x, k0);
        const int y0 = k0 + L0 * lj;  // lane's first output row; element (m, q) adds L0 * out_dy
        float2* out = dst + (size_t)up * N * N + (size_t)y0 * N + x;
        auto emit = [&](int m, int q, float2 val) {
            const int dy = CT::out_dy(m, q);
            const float s = perm_sign(x, y0 + L0 * dy);
            out[(size_t)L0 * dy * N] = make_float2(val.x * s, val.y * s);
        };
        E::run_regs(cur, lds, twl, emit);
#pragma unroll
        for (int i = 0; i < kElems; ++i) cur[i] = nxt[i];
        __syncthreads();
    }
}

// ------------------------------------------- folded columns (N = 2048 / 4096)
// The column transform at N = F L (F = 2 / 4) split by decimation in frequency:
//   X[F m + b] = sum_{n < L} z_b[n] w_L^(n m),   z_b[n] = w_N^(n b) sum_{r < F} a[n + L r] w_F^(r b).
// k_rowsf transforms rows n + L r (r < F) of one unit-plane, folds the F results column by column into
// z_b[n] and stores z_b at row b L + n of the scratch (sub-plane b);
// k_colsf runs L-point column tiles over the scratch's sub-planes -- the N = 2048 column shape at F = 2
// (8-column halves, XCD-paired: 64-byte pieces of 128-byte lines), the N = 1024 one at F = 4 (8 or 16
// wide) -- and writes row F m + b of the plane, permuted.  The 4-column tiles of a whole 4096-point
// column (32-byte pieces) are not needed.  At 4096 the default is F = 2 (ocean_abi.cpp, OCEAN_FOLD_F).
#ifndef OCEAN_ROWSF_WPEU
#define OCEAN_ROWSF_WPEU 0  // waves per SIMD k_rowsf is compiled for (0: the compiler's choice; A/B builds)
#endif
#if OCEAN_ROWSF_WPEU
#define ROWSF_WPEU __attribute__((amdgpu_waves_per_eu(OCEAN_ROWSF_WPEU)))
#else
#define ROWSF_WPEU
#endif

// k_rowsf: a one-row engine (N / 16 lanes); item n runs its F rows n + L r back to back, in the order
// r = 0, 2, 1, 3 (F = 4) or 0, 1 (F = 2), with the next row's loads in flight across each row's stages.
// A lane's last-stage outputs sit at the same columns x for every row, so the fold is a radix-F
// butterfly in registers, formed incrementally: (a0 + a2, a0 - a2) after row 2, a1 held, then
// z_0 = s0 + s1, z_2 = s0 - s1, z_1 = d0 + i d1, z_3 = d0 - i d1 with s1, d1 = a1 +- a3.
template <int N, int F>
__global__ __launch_bounds__(N / kElems) ROWSF_WPEU void k_rowsf(const float2* __restrict__ plane, float2* __restrict__ scratch,
                                                      int items, const float2* __restrict__ tw) {
    constexpr int L = N / F;
    static_assert(F == 2 || F == 4, "fold of 2 or 4 rows");
    using TW = StageTwLds<N>;
    using E = Engine<N, 1, false, true, 16, TW>;
    constexpr int T = E::THREADS;
    static_assert(kElems == E::R0, "one stage-0 butterfly per lane");
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    TW::load(twl, tw, threadIdx.x, T);
    const float2* tws = TW::table(twl, tw);
    const int j = (int)threadIdx.x;
    // sub-step k of item it: row n + L r(k), r = 0, 2, 1, 3 (F = 4) / 0, 1 (F = 2)
    auto row_of = [&](int it, int k) {
        const int up = it / L, n = it - up * L;
        const int r = F == 4 ? ((k & 1) << 1 | (k >> 1)) : k;
        return (size_t)up * N * N + (size_t)(n + L * r) * N;
    };
    auto load = [&](int it, int k, float2 (&d)[kElems]) {
        const Win w = make_win(plane + row_of(it, k), (unsigned)(N * 8));
#pragma unroll
        for (int q = 0; q < kElems; ++q) d[q] = bload2(w, j * 8, q * (N / kElems) * 8);
    };
    float2 cur[kElems], nxt[kElems];
    float2 h0[kElems], h1[kElems], h2[F == 4 ? kElems : 1];
    int it = blockIdx.x;
    if (it < items) load(it, 0, cur);
    __syncthreads();  // twiddle table
    for (; it < items; it += gridDim.x) {
        const int up = it / L, n = it - up * L;
        float2* dst = scratch + (size_t)up * N * N + (size_t)n * N;  // row b L + n holds z_b w_N^(n b)
        float2 wf[F];
#pragma unroll
        for (int b = 1; b < F; ++b) wf[b] = tw[n * b];  // n b < N
#pragma unroll
        for (int k = 0; k < F; ++k) {
            if (k + 1 < F) load(it, k + 1, nxt);
            else if (it + (int)gridDim.x < items) load(it + gridDim.x, 0, nxt);
            // the fold runs on each last-stage value as it is emitted; the last row's values complete it
            auto emit = [&](int m, int q, float2 val) {
                const int i = m * E::RL + q;
                if (k == 0) {
                    h0[i] = val;                        // a0
                } else if (F == 4 && k == 1) {
                    h1[i] = csub(h0[i], val);           // d0 = a0 - a2
                    h0[i] = cadd(h0[i], val);           // s0 = a0 + a2
                } else if (F == 4 && k == 2) {
                    h2[i] = val;                        // a1
                } else {
                    int bb, jj;
                    E::template bj<E::RL>(j + m * T, bb, jj);
                    const int x = jj + q * (N / E::RL);
                    if constexpr (F == 4) {
                        const float2 s1 = cadd(h2[i], val), d1 = cmul_i(csub(h2[i], val));
                        dst[x] = cadd(h0[i], s1);
                        dst[(size_t)1 * L * N + x] = cmul(cadd(h1[i], d1), wf[1]);
                        dst[(size_t)2 * L * N + x] = cmul(csub(h0[i], s1), wf[2]);
                        dst[(size_t)3 * L * N + x] = cmul(csub(h1[i], d1), wf[3]);
                    } else {
                        dst[x] = cadd(h0[i], val);
                        dst[(size_t)L * N + x] = cmul(csub(h0[i], val), wf[1]);
                    }
                }
            };
            E::run_regs(cur, lds, tws, emit);
#pragma unroll
            for (int i = 0; i < kElems; ++i) cur[i] = nxt[i];
            __syncthreads();  // the image is free for the next row's stage 0
        }
    }
}

// item = (unit-plane, sub-plane b, W-column tile); G > 1 groups the pieces of 16-column tiles on one
// XCD as k_cols2 does.
template <int N, int F, int W, int G>
__global__ __launch_bounds__(W * (N / F) / kElems) void k_colsf(const float2* __restrict__ scratch,
                                                                float2* __restrict__ plane, int items,
                                                                const float2* __restrict__ tw) {
    constexpr int L = N / F;
    using CT = ColTile<L, W>;  // geometry only: lanes, in_dy / out_dy
    using TW = OpSubTw<L, N>;
    using E = Engine<L, W, true, Engine<L, W, true, false>::seq_pad_ok(), 16, TW>;
    static_assert(E::THREADS == CT::T && E::R0 == CT::R0 && E::RL == CT::RL, "tile geometry");
    constexpr int T = E::THREADS;
    constexpr int TILES = N / W;  // column tiles per sub-plane
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    TW::load(twl, tw, threadIdx.x, T);
    const int lb = CT::lane_b(), lj = CT::lane_j();
    const int voff = (lj * N + lb) * 8;          // input element (lb, n = lj) of a sub-plane tile
    const int ooff = (F * lj * N + lb) * 8;      // output element (lb, y = F lj) from the tile's row b
    auto tile_of = [&](int item) {
        if constexpr (G > 1) return (item & ~(8 * G - 1)) + G * (item & 7) + ((item >> 3) & (G - 1));
        else return item;
    };
    auto decode = [&](int item, int& up, int& b, int& x0) {
        const int t = tile_of(item);
        up = t / (F * TILES);
        const int r = t - up * F * TILES;
        b = r / TILES;
        x0 = (r - b * TILES) * W;
    };
    float2 cur[kElems], nxt[kElems];
    auto load = [&](int item, float2 (&d)[kElems]) {
        int up, b, x0;
        decode(item, up, b, x0);
        const size_t o = (size_t)up * N * N + (size_t)b * L * N + x0;
        const Win w = make_win(scratch + o, (unsigned)(((size_t)L * N - x0) * 8));
#pragma unroll
        for (int i = 0; i < kElems; ++i) d[i] = bload2(w, voff, CT::in_dy(i) * N * 8);
    };
    int item = blockIdx.x;
    if (item < items) load(item, cur);
    __syncthreads();
    for (; item < items; item += gridDim.x) {
        const int next = item + gridDim.x;
        if (next < items) load(next, nxt);
        int up, b, x0;
        decode(item, up, b, x0);
        const Win w = make_win(plane + (size_t)up * N * N + (size_t)b * N + x0, 0);
        auto emit = [&](int m, int q, float2 val) {
            const int dy = CT::out_dy(m, q);
            const float s = perm_sign(x0 + lb, F * (lj + dy) + b);
            gstore2(make_float2(val.x * s, val.y * s), w, ooff, F * dy * N * 8);
        };
        E::run_regs(cur, lds, twl, emit);
#pragma unroll
        for (int i = 0; i < kElems; ++i) cur[i] = nxt[i];
        __syncthreads();
    }
}

// --------------------------------------------------------------- launch
template <class K>
int persistent_grid(K kernel, int threads, int items) {
    const int g = device_cus() * resident_per_cu((const void*)kernel, threads);
    return items < g ? items : g;
}

template <template <int> class F, class... A>
hipError_t dispatch_n(int n, A... a) {
    switch (n) {
        case 16: return F<16>::go(a...);
        case 32: return F<32>::go(a...);
        case 64: return F<64>::go(a...);
        case 128: return F<128>::go(a...);
        case 256: return F<256>::go(a...);
        case 512: return F<512>::go(a...);
        case 1024: return F<1024>::go(a...);
        case 2048: return F<2048>::go(a...);
        case 4096: return F<4096>::go(a...);
    }
    return hipErrorInvalidValue;
}

// In-place row / column launches over `ups` consecutive unit-planes at `base` (plane p of unit u is
// unit-plane p * U + u of the one plane allocation).
template <int N>
struct Rows2 {
    template <int B>
    static hipError_t go_b(const DevView* v, float2* base, int ups, hipStream_t s) {
        constexpr int T = B * N / kElems;
        const int total = ups * N;
        const int items = (total + B - 1) / B;
        const int g = persistent_grid(k_rows2<N, B>, T, items);
        launch((k_rows2<N, B>), dim3(g), dim3(T), 0, s, (const float2*)base, base, total, v->tw);
        return hipGetLastError();
    }
    static hipError_t go(const DevView* v, float2* base, int ups, hipStream_t s) {
        return go_b<rows_per_item(N)>(v, base, ups, s);
    }
};
template <int N>
struct Cols2 {
    template <int W, int G>
    static hipError_t go_w(const DevView* v, float2* base, int ups, hipStream_t s) {
        constexpr int T = W * N / kElems;
        const int items = ups * (N / W);
        int g = persistent_grid(k_cols2<N, W, G>, T, items);
        if (G > 1) g -= g % (8 * G);  // pieces of a tile on blocks b, b + 8, ... at every step of the item loop
        launch((k_cols2<N, W, G>), dim3(g), dim3(T), 0, s, base, items, v->tw);
        return hipGetLastError();
    }
    static hipError_t go(const DevView* v, float2* base, int ups, hipStream_t s) {
        if constexpr (N == 1024) {
            // default: 8-column halves paired on one XCD (45.6 against 49.7 us for 4 x 1024^2 x 4 planes);
            // OCEAN_COLS2_XP=0 selects the 16-column tiles (A/B)
            static const int xp = std::getenv("OCEAN_COLS2_XP") ? std::atoi(std::getenv("OCEAN_COLS2_XP")) : 1;
            if (xp) return go_w<8, 2>(v, base, ups, s);
        }
        if constexpr (N >= 2048) {
            // default: column pieces of 16-column tiles grouped on one XCD -- 8-column halves at 2048,
            // 4-column quarters at 4096 (whole columns in LDS: 128 KiB) -- 0.65 / 0.57 of peak against
            // 0.25 / 0.26 ungrouped (4 columns, 32-byte row pieces).  OCEAN_COLS2_XQ: 0 ungrouped, 1 4 x 4,
            // 2 2 x 8, 3 8 x 2 (2048) -- A/B
            static const int xq = std::getenv("OCEAN_COLS2_XQ") ? std::atoi(std::getenv("OCEAN_COLS2_XQ")) : -1;
            if (xq == 1 || (xq < 0 && N == 4096)) return go_w<4, 4>(v, base, ups, s);
            if (xq == 2) return go_w<2, 8>(v, base, ups, s);
            if constexpr (N == 2048)
                if (xq == 3 || xq < 0) return go_w<8, 2>(v, base, ups, s);
        }
        return go_w<cols2_w(N), 1>(v, base, ups, s);
    }
};
// Four-step operator for N = 2048 / 4096 over `ups` consecutive unit-planes at `planes` (one
// allocation: plane p of unit u is unit-plane p * U + u), through `scratch` (>= ups unit-planes).
template <int N>
struct Op4 {
    template <int B>
    static hipError_t rows_to(const DevView* v, float2* planes, int ups, float2* scratch, hipStream_t s) {
        constexpr int T = B * N / kElems;
        const int total = ups * N;
        const int items = (total + B - 1) / B;
        const int g = persistent_grid(k_rows2<N, B>, T, items);
        launch((k_rows2<N, B>), dim3(g), dim3(T), 0, s, (const float2*)planes, scratch, total, v->tw);
        return hipGetLastError();
    }
    static hipError_t go(const DevView* v, float2* planes, int ups, float2* scratch, int part, hipStream_t s) {
        if constexpr (N < 2048) {
            return hipErrorInvalidValue;
        } else {
            if (part == 0) {  // rows: planes -> scratch
                static const int rb = std::getenv("OCEAN_OP_ROWS_B") ? std::atoi(std::getenv("OCEAN_OP_ROWS_B")) : 1;
                if (rb == 2) return rows_to<2>(v, planes, ups, scratch, s);  // A/B: two rows per workgroup
                return rows_to<rows_per_item(N)>(v, planes, ups, scratch, s);
            } else if (part == 1) {  // C1 in place on the scratch
                constexpr int T = kOpSeq * (N / kOpL1) / kElems;
                const int items = ups * (N / kOpW) * (kOpL1 / kOpBlk);
                const int g = persistent_grid(k_opc1<N>, T, items);
                launch((k_opc1<N>), dim3(g), dim3(T), 0, s, scratch, items, v->tw);
            } else {  // C2: scratch -> planes
                constexpr int T = kOpSeq * kOpL1 / kElems;
                const int items = ups * (N / kOpW) * ((N / kOpL1) / kOpBlk);
                const int g = persistent_grid(k_opc2<N>, T, items);
                launch((k_opc2<N>), dim3(g), dim3(T), 0, s, (const float2*)scratch, planes, items, v->tw);
            }
            return hipGetLastError();
        }
    }
};

// Folded operator for N = 2048 / 4096 over `ups` consecutive unit-planes: part 0 = k_rowsf (planes ->
// scratch sub-planes), part 1 / 2 = k_colsf on 8 / 16-column tiles (scratch -> planes, permuted).
template <int N>
struct OpFold {
    template <int F, int W, int G>
    static hipError_t cols(const DevView* v, float2* planes, int ups, const float2* scratch, hipStream_t s) {
        constexpr int T = W * (N / F) / kElems;
        const int items = ups * F * (N / W);
        int g = persistent_grid(k_colsf<N, F, W, G>, T, items);
        if (G > 1) g -= g % (8 * G);
        launch((k_colsf<N, F, W, G>), dim3(g), dim3(T), 0, s, scratch, planes, items, v->tw);
        return hipGetLastError();
    }
    template <int F>
    static hipError_t rows(const DevView* v, float2* planes, int ups, float2* scratch, hipStream_t s) {
        constexpr int T = N / kElems;
        const int items = ups * (N / F);
        const int g = persistent_grid(k_rowsf<N, F>, T, items);
        launch((k_rowsf<N, F>), dim3(g), dim3(T), 0, s, (const float2*)planes, scratch, items, v->tw);
        return hipGetLastError();
    }
    static hipError_t go(const DevView* v, float2* planes, int ups, float2* scratch, int part, int fold,
                         hipStream_t s) {
        if constexpr (N == 2048) {
            if (fold != 2) return hipErrorInvalidValue;
            if (part == 0) return rows<2>(v, planes, ups, scratch, s);
            if (part == 2) return cols<2, 16, 1>(v, planes, ups, scratch, s);
            return cols<2, 8, 2>(v, planes, ups, scratch, s);
        } else if constexpr (N == 4096) {
            if (fold == 2) {  // 2048-point columns: 8-column halves paired on one XCD (the N = 2048 shape)
                if (part == 0) return rows<2>(v, planes, ups, scratch, s);
                return cols<2, 8, 2>(v, planes, ups, scratch, s);
            }
            if (fold != 4) return hipErrorInvalidValue;
            if (part == 0) return rows<4>(v, planes, ups, scratch, s);
            // part 1: 8-column halves of 16-column tiles paired on one XCD (k_cols2 at N = 1024);
            // part 2: whole 16-column tiles (A/B, OCEAN_FOLD_COLS=16)
            if (part == 2) return cols<4, 16, 1>(v, planes, ups, scratch, s);
            return cols<4, 8, 2>(v, planes, ups, scratch, s);
        } else {
            return hipErrorInvalidValue;
        }
    }
};

template <int N>
struct StageTwCount {
    static hipError_t go(size_t* out) {
        *out = (size_t)StageTw<N, 16>::off(n_stages(N, 16)) + (size_t)StageTw<N, 8>::off(n_stages(N, 8)) +
               (size_t)StageTw<N, 4>::off(n_stages(N, 4));
        return hipSuccess;
    }
};

}  // namespace

size_t stage_twiddle_entries(int n) {
    size_t e = 0;
    (void)dispatch_n<StageTwCount>(n, &e);
    return e;
}

hipError_t launch_ifft_rows_v2(const DevView& v, float2* base, int ups, hipStream_t s) {
    return dispatch_n<Rows2>(v.n, &v, base, ups, s);
}
hipError_t launch_ifft_cols_v2(const DevView& v, float2* base, int ups, hipStream_t s) {
    return dispatch_n<Cols2>(v.n, &v, base, ups, s);
}
hipError_t launch_ifft_four_step(const DevView& v, float2* planes, int ups, float2* scratch, int part, hipStream_t s) {
    if (v.n != 2048 && v.n != 4096) return hipErrorInvalidValue;
    return v.n == 2048 ? Op4<2048>::go(&v, planes, ups, scratch, part, s) : Op4<4096>::go(&v, planes, ups, scratch, part, s);
}
hipError_t launch_ifft_fold(const DevView& v, float2* planes, int ups, float2* scratch, int part, int fold,
                            hipStream_t s) {
    if (v.n != 2048 && v.n != 4096) return hipErrorInvalidValue;
    return v.n == 2048 ? OpFold<2048>::go(&v, planes, ups, scratch, part, fold, s)
                       : OpFold<4096>::go(&v, planes, ups, scratch, part, fold, s);
}

}  // namespace ocean
