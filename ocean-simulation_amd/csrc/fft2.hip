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
constexpr int rows_per_item(int N) { return N >= 1024 ? 4 : 4096 / N; }

// Standalone row pass, in place: item = B consecutive rows of the flattened
// [unit][y] row list of one plane.
template <int N, int B = rows_per_item(N)>
__global__ __launch_bounds__(B * N / kElems) void k_rows2(float2* __restrict__ plane, int total_rows,
                                                         const float2* __restrict__ tw) {
    using E = Engine<N, B, false, true>;
    using TW = StageTw<N>;
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
        const Win w = make_win(plane + (size_t)item * B * N, 0);
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

// XP (W = 8 at N = 1024): the two 8-column halves of a 16-column tile go to items i and i + 8,
// which blocks b and b + 8 -- one XCD under round-robin placement (speed only, never correctness)
// -- take at the same time, so each 128-byte line is fetched and written back through one L2.
template <int N, int W_ = cols2_w(N), bool XP = false>
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
        if constexpr (XP) return (item & ~15) + 2 * (item & 7) + ((item >> 3) & 1);
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

template <int N>
struct Rows2 {
    template <int B>
    static hipError_t go_b(const DevView* v, int p, int np, hipStream_t s) {
        constexpr int T = B * N / kElems;
        const int total = np * v->units * N;
        const int items = (total + B - 1) / B;
        const int g = persistent_grid(k_rows2<N, B>, T, items);
        launch((k_rows2<N, B>), dim3(g), dim3(T), 0, s, v->plane[p], total, v->tw);
        return hipGetLastError();
    }
    static hipError_t go(const DevView* v, int p, int np, hipStream_t s) {
        return go_b<rows_per_item(N)>(v, p, np, s);
    }
};
template <int N>
struct Cols2 {
    template <int W, bool XP>
    static hipError_t go_w(const DevView* v, int p, int np, hipStream_t s) {
        constexpr int T = W * N / kElems;
        const int items = np * v->units * (N / W);
        int g = persistent_grid(k_cols2<N, W, XP>, T, items);
        if (XP) g -= g % 16;  // halves of a tile on blocks b, b + 8 at every step of the item loop
        launch((k_cols2<N, W, XP>), dim3(g), dim3(T), 0, s, v->plane[p], items, v->tw);
        return hipGetLastError();
    }
    static hipError_t go(const DevView* v, int p, int np, hipStream_t s) {
        if constexpr (N == 1024) {
            // default: 8-column halves paired on one XCD (45.6 against 49.7 us for 4 x 1024^2 x 4 planes);
            // OCEAN_COLS2_XP=0 selects the 16-column tiles (A/B)
            static const int xp = std::getenv("OCEAN_COLS2_XP") ? std::atoi(std::getenv("OCEAN_COLS2_XP")) : 1;
            if (xp) return go_w<8, true>(v, p, np, s);
        }
        return go_w<cols2_w(N), false>(v, p, np, s);
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

hipError_t launch_ifft_rows_v2(const DevView& v, int p, int np, hipStream_t s) {
    return dispatch_n<Rows2>(v.n, &v, p, np, s);
}
hipError_t launch_ifft_cols_v2(const DevView& v, int p, int np, hipStream_t s) {
    return dispatch_n<Cols2>(v.n, &v, p, np, s);
}

}  // namespace ocean
