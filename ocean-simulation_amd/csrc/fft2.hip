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
#include "fft_engine.h"

namespace ocean {
namespace {

// -------------------------------------------------------------- kernels
// rows per workgroup of k_rows2: 4 at N = 1024 (1024 lanes); one row (256 lanes, 3 workgroups per CU)
// at N = 2048 / 4096, where a 4-row image (128 / 256 KiB) held one workgroup per CU
constexpr int rows_per_item(int N) { return N >= 2048 ? 1 : (N >= 1024 ? 4 : 4096 / N); }

// Standalone row pass, in place: item = B consecutive rows of the flattened
// [unit][y] row list of one plane.
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
// default is W = 8 with XCD-paired halves (G = 2 below): 2 workgroups per CU instead of 1, and every
// 128-byte line still moves through one L2.
constexpr int cols2_w(int N) { return N == 1024 ? 16 : col_tile(N); }

// G > 1 (XCD grouping): the G W-column pieces of a (G W)-column tile go to items i, i + 8, ...,
// i + 8 (G - 1), which blocks b, b + 8, ... -- one XCD under round-robin placement (speed only, never
// correctness) -- take at the same time, so each 128-byte line is fetched and written back through one
// L2.  G = 2, W = 8 at N = 1024 and 2048.
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

// ------------------------------------------------- folded columns (N = 4096)
// The column transform at N = F L (F = 2) split by decimation in frequency:
//   X[F m + b] = sum_{n < L} z_b[n] w_L^(n m),   z_b[n] = w_N^(n b) (a[n] + (-1)^b a[n + L]).
// Both launches work in place on the planes.  k_rowsf transforms rows n and n + L of one unit-plane,
// folds the two results column by column into z_b[n] and stores z_b at row b L + n (sub-plane b);
// k_colsf_ip runs L-point column tiles over both sub-planes -- the N = 2048 column shape (8-column
// halves, XCD-paired: 64-byte pieces of 128-byte lines) -- and writes row F m + b, permuted.  The
// 4-column tiles of a whole 4096-point column (32-byte pieces, 0.57 of peak) are not needed, and the
// round-4 form through a scratch plane set (twice the cache footprint per chunk) is gone
// (docs/MEASUREMENTS.md sections 3 and 8).

// k_rowsf: a one-row engine (N / 16 lanes); item n runs its rows n, n + L back to back with the next
// row's loads in flight across each row's stages.  A lane's last-stage outputs sit at the same columns
// x for both rows, so the fold is a radix-2 butterfly in registers as the second row's values are
// emitted: z_0 = a0 + a1, z_1 = (a0 - a1) w_N^n.  An item writes only the two rows it has read (z_0 to
// row n, z_1 to row n + L), after reading both.
template <int N>
__global__ __launch_bounds__(N / kElems) void k_rowsf(float2* plane, int items, const float2* __restrict__ tw) {
    constexpr int F = 2, L = N / F;
    using TW = StageTwLds<N>;
    using E = Engine<N, 1, false, true, 16, TW>;
    constexpr int T = E::THREADS;
    static_assert(kElems == E::R0, "one stage-0 butterfly per lane");
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    TW::load(twl, tw, threadIdx.x, T);
    const float2* tws = TW::table(twl, tw);
    const int j = (int)threadIdx.x;
    auto load = [&](int it, int k, float2 (&d)[kElems]) {
        const int up = it / L, n = it - up * L;
        const Win w = make_win(plane + (size_t)up * N * N + (size_t)(n + L * k) * N, (unsigned)(N * 8));
#pragma unroll
        for (int q = 0; q < kElems; ++q) d[q] = bload2(w, j * 8, q * (N / kElems) * 8);
    };
    float2 cur[kElems], nxt[kElems], h0[kElems];
    int it = blockIdx.x;
    if (it < items) load(it, 0, cur);
    __syncthreads();  // twiddle table
    for (; it < items; it += gridDim.x) {
        const int up = it / L, n = it - up * L;
        float2* dst = plane + (size_t)up * N * N + (size_t)n * N;  // row b L + n holds z_b
        const float2 wf = tw[n];                                      // w_N^n
#pragma unroll
        for (int k = 0; k < F; ++k) {
            if (k + 1 < F) load(it, k + 1, nxt);
            else if (it + (int)gridDim.x < items) load(it + gridDim.x, 0, nxt);
            auto emit = [&](int m, int q, float2 val) {
                const int i = m * E::RL + q;
                if (k == 0) {
                    h0[i] = val;  // a0
                } else {
                    int bb, jj;
                    E::template bj<E::RL>(j + m * T, bb, jj);
                    const int x = jj + q * (N / E::RL);
                    dst[x] = cadd(h0[i], val);
                    dst[(size_t)L * N + x] = cmul(csub(h0[i], val), wf);
                }
            };
            E::run_regs(cur, lds, tws, emit);
#pragma unroll
            for (int i = 0; i < kElems; ++i) cur[i] = nxt[i];
            __syncthreads();  // the image is free for the next row's stage 0
        }
    }
}

// The in-place column launch over the row launch's sub-planes (k_rowsf: z_b at rows b L + n of the plane
// itself).  Sub-plane b's outputs go to rows F m + b, which for m >= L/2 are rows of sub-plane 1: so item =
// (unit-plane, W-column tile) transforms sub-plane 0 then sub-plane 1 of its columns, writes sub-plane 0's
// outputs m < L/2 as they come (rows 2m < L, already read), holds the other half (8 values per lane) in
// registers until every lane has read sub-plane 1's tile (the barrier after its stage 0), then writes
// them.  A chunk's cache footprint is its own planes.  Loads are issued into the stage-0 registers once
// their values are in the LDS image (sub-plane 1 during sub-plane 0's stages, the next item's sub-plane 0
// during sub-plane 1's), so no second register buffer is needed for the prefetch.  G > 1 groups the
// 8-column halves of 16-column tiles on one XCD as k_cols2 does.  The outputs stored as they come (three
// quarters) are nontemporal, the held quarter default-policy: the next chunk's row launch then reads its
// planes past a cache that the finished chunk's outputs do not fill (rows 0.71 -> 0.77, columns
// unchanged at 0.65, wall 0.68 -> 0.70; all nontemporal: columns 0.62, wall 0.69; docs/MEASUREMENTS.md
// section 8).
template <int N, int W, int G>
__global__ __launch_bounds__(W * (N / 2) / kElems) void k_colsf_ip(float2* plane, int items,
                                                                   const float2* __restrict__ tw) {
    constexpr int F = 2, L = N / F;
    using CT = ColTile<L, W>;  // geometry only: lanes, in_dy / out_dy
    using TW = SubTw<L, N>;
    using E = Engine<L, W, true, Engine<L, W, true, false>::seq_pad_ok(), 16, TW>;
    static_assert(E::THREADS == CT::T && E::R0 == CT::R0 && E::RL == CT::RL, "tile geometry");
    constexpr int T = E::THREADS;
    constexpr int TILES = N / W;        // column tiles per unit-plane
    constexpr int BF = kElems / E::RL;  // last-stage butterflies per lane
    constexpr int HALF_Q = E::RL / 2;   // q >= HALF_Q: output m >= L/2 (out_dy's q stride is L / RL)
    static_assert(CT::out_dy(0, HALF_Q) == L / 2 && (T / W) * BF <= L / E::RL, "held half = q >= RL / 2");
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    TW::load(twl, tw, threadIdx.x, T);
    const int lb = CT::lane_b(), lj = CT::lane_j();
    const int voff = (lj * N + lb) * 8;      // input element (lb, n = lj) of a sub-plane tile
    const int ooff = (F * lj * N + lb) * 8;  // output element (lb, y = F lj) of the tile's rows
    auto tile_of = [&](int item) {
        if constexpr (G > 1) return (item & ~(8 * G - 1)) + G * (item & 7) + ((item >> 3) & (G - 1));
        else return item;
    };
    auto decode = [&](int item, int& up, int& x0) {
        const int t = tile_of(item);
        up = t / TILES;
        x0 = (t - up * TILES) * W;
    };
    float2 cur[kElems];
    float2 held[BF * (E::RL - HALF_Q)];  // sub-plane 0's outputs m >= L/2, sign applied
    auto load = [&](int item, int b) {
        int up, x0;
        decode(item, up, x0);
        const size_t o = (size_t)up * N * N + (size_t)b * L * N + x0;
        const Win w = make_win(plane + o, (unsigned)(((size_t)L * N - x0) * 8));
#pragma unroll
        for (int i = 0; i < kElems; ++i) cur[i] = bload2(w, voff, CT::in_dy(i) * N * 8);
    };
    int item = blockIdx.x;
    if (item < items) load(item, 0);
    __syncthreads();  // twiddle table
    for (; item < items; item += gridDim.x) {
        int up, x0;
        decode(item, up, x0);
        const Win w = make_win(plane + (size_t)up * N * N + x0, 0);
#pragma unroll
        for (int b = 0; b < F; ++b) {
#pragma unroll
            for (int m = 0; m < kElems / E::R0; ++m) {
                Idft<E::R0>::run(&cur[m * E::R0]);
                E::stage0_store(lds, m, &cur[m * E::R0]);
            }
            __syncthreads();  // the image holds sub-plane b; every lane has read sub-plane b's tile
            if (b == 0) {
                load(item, 1);  // sub-plane 1, in flight across sub-plane 0's stages
            } else {
                if (item + (int)gridDim.x < items) load(item + gridDim.x, 0);  // the next item's sub-plane 0
                // sub-plane 1 is read: sub-plane 0's outputs m >= L/2 may overwrite its rows now
#pragma unroll
                for (int m = 0; m < BF; ++m)
#pragma unroll
                    for (int q = HALF_Q; q < E::RL; ++q)
                        gstore2(held[m * (E::RL - HALF_Q) + q - HALF_Q], w, ooff, F * CT::out_dy(m, q) * N * 8);
            }
            auto emit = [&](int m, int q, float2 val) {
                const int dy = CT::out_dy(m, q);
                const float s = perm_sign(x0 + lb, F * (lj + dy) + b);
                const float2 o = make_float2(val.x * s, val.y * s);
                if (b == 0 && q >= HALF_Q) held[m * (E::RL - HALF_Q) + q - HALF_Q] = o;
                else gstore2_nt(o, w, ooff + b * N * 8, F * dy * N * 8);
            };
            E::template stages_from<1>(lds, twl, emit);
            __syncthreads();  // the image is free for the next stage 0
        }
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
        // 8-column halves paired on one XCD at N = 1024 (45.6 against 49.7 us for 4 x 1024^2 x 4 planes
        // on whole 16-column tiles) and 2048 (0.65 against 0.25 of peak ungrouped); N = 4096 runs the
        // folded columns instead (OpFold)
        if constexpr (N == 1024 || N == 2048) return go_w<8, 2>(v, base, ups, s);
        else if constexpr (N == 4096) return hipErrorInvalidValue;
        else return go_w<cols2_w(N), 1>(v, base, ups, s);
    }
};

// Folded operator for N = 4096 over `ups` consecutive unit-planes, in place: part 0 = k_rowsf (rows + fold
// onto the planes' own rows), part 1 = k_colsf_ip (both sub-planes of an 8-column tile per item, permuted).
struct OpFold {
    static constexpr int N = 4096, F = 2, W = 8, G = 2;  // 4-column tiles: 0.48 (docs/MEASUREMENTS.md section 8)
    static hipError_t go(const DevView* v, float2* planes, int ups, int part, hipStream_t s) {
        if (part == 0) {
            constexpr int T = N / kElems;
            const int items = ups * (N / F);
            const int g = persistent_grid(k_rowsf<N>, T, items);
            launch((k_rowsf<N>), dim3(g), dim3(T), 0, s, planes, items, v->tw);
        } else {
            constexpr int T = W * (N / F) / kElems;
            const int items = ups * (N / W);
            int g = persistent_grid(k_colsf_ip<N, W, G>, T, items);
            g -= g % (8 * G);  // the pieces of a tile on blocks b, b + 8, ... at every step of the item loop
            launch((k_colsf_ip<N, W, G>), dim3(g), dim3(T), 0, s, planes, items, v->tw);
        }
        return hipGetLastError();
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
hipError_t launch_ifft_fold(const DevView& v, float2* planes, int ups, int part, hipStream_t s) {
    if (v.n != OpFold::N) return hipErrorInvalidValue;
    return OpFold::go(&v, planes, ups, part, s);
}

}  // namespace ocean
