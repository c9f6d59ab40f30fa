// v2 FFT kernels for gfx950: persistent workgroups, software-pipelined
// loads, LDS-resident per-stage twiddles, compile-time LDS offsets.
//
// Same transforms as fft.hip (see its header for the reference mapping and
// the Stockham formulation); what changes is how the work meets the machine:
//  * persistent grid (CUs x resident workgroups); each workgroup walks items
//    (rows / column tiles) with stride gridDim.x;
//  * the NEXT plane's (or next item's) global loads are issued into registers
//    before the current plane's FFT stages and stores (vmcnt counts loads and
//    stores in issue order, so the prefetch goes out first);
//  * global loads use buffer_load with one 32-bit voffset per lane and the
//    per-element stride in the scalar soffset; stores are plain global stores
//    (see the note at "memory ops");
//  * every LDS access of a butterfly is (per-lane base) + (compile-time
//    offset): the row layout is padded one complex per 16 and all Stockham
//    strides are multiples of 16 there, the column-tile layout is unpadded
//    ([y][W], b-fastest lanes keep it at most 2-way conflicted);
//  * twiddles come from per-stage tables laid out [k][r] (the R-1 twiddles of
//    a butterfly are contiguous), copied to LDS when they fit;
//  * pass B keeps at most two values per texel live across planes
//    (plane order DyDxz, DxDz, DxxDzz, DyxDyz).
#include "fft_engine.h"
#include "spectrum_math.h"

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
// W = 16 at N = 1024 (128-byte row segments; 1024 lanes), col_tile(N) otherwise.
constexpr int cols2_w(int N) { return N == 1024 ? 16 : col_tile(N); }

template <int N>
__global__ __launch_bounds__(cols2_w(N) * N / kElems) void k_cols2(float2* __restrict__ plane, int items,
                                                                  const float2* __restrict__ tw) {
    using CT = ColTile<N, cols2_w(N)>;
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
    auto win = [&](int item) {
        const int u = item / CT::tiles, x0 = (item - u * CT::tiles) * W;
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
        const int x0 = (item % CT::tiles) * W;
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

// Fused pass A: evolve + row IFFT of the P planes.  Item = RB consecutive
// rows; LDS sequence b = p * RB + row.  Each lane evolves TPT = 16 / P texels.
template <int N, int P>
constexpr int pa_rows2() { return N >= 1024 ? 1 : 1024 / N; }

template <int N, int P>
__global__ __launch_bounds__((pa_rows2<N, P>() * P * N / kElems)) void k_pass_a2(DevView v, float time,
                                                                                 int total_rows) {
    constexpr int RB = pa_rows2<N, P>();
    constexpr int B = RB * P;
    using E = Engine<N, B, false, true>;
    using TW = StageTw<N>;
    constexpr int T = E::THREADS;
    constexpr int TPT = RB * N / T;
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    TW::load(twl, v.tw, threadIdx.x, T);
    const float2* tws = TW::table(twl, v.tw);
    const int items = (total_rows + RB - 1) / RB;
    float4 h[TPT], w[TPT], hn[TPT], wn[TPT];
    auto load = [&](int item, float4 (&hh)[TPT], float4 (&ww)[TPT]) {
        const int rows = min(RB, total_rows - item * RB);
        const Win rh = make_win(v.h0 + (size_t)item * RB * N, (unsigned)(rows * N * 16));
        const Win rw = make_win(v.waves + (size_t)item * RB * N, (unsigned)(rows * N * 16));
#pragma unroll
        for (int k = 0; k < TPT; ++k) {  // rows past the end read 0 (buffer range check)
            hh[k] = bload4(rh, (int)threadIdx.x * 16, k * T * 16);
            ww[k] = bload4(rw, (int)threadIdx.x * 16, k * T * 16);
        }
    };
    int item = blockIdx.x;
    if (item < items) load(item, h, w);
    for (; item < items; item += gridDim.x) {
        const int next = item + gridDim.x;
        if (next < items) load(next, hn, wn);
#pragma unroll
        for (int k = 0; k < TPT; ++k) {
            const int e = (int)threadIdx.x + k * T;
            const int rr = e / N, x = e % N;
            const Planes4 o = evolve_texel(h[k], w[k], time);
            // sequence p * RB + rr starts at raw index (p * RB + rr) * N, a multiple of 16
            float2* dst = lds + E::lidx(rr, x);
#pragma unroll
            for (int p = 0; p < P; ++p) dst[p * padded(RB * N)] = o.p[p];
        }
        __syncthreads();
        // planes are one allocation: plane p at p * plane_stride
        const Win wp = make_win(v.plane[0] + (size_t)item * RB * N, 0);
        const int pstride8 = (int)(v.plane_stride * 8);
        auto emit = [&](int m, int q, float2 val) {
            int b, j;
            E::template bj<E::RL>((int)threadIdx.x + m * T, b, j);
            const int p = b / RB, rr = b % RB;
            if (item * RB + rr < total_rows) gstore2(val, wp, p * pstride8 + (rr * N + j) * 8, q * (N / E::RL) * 8);
        };
        E::run_lds(lds, tws, emit);
#pragma unroll
        for (int k = 0; k < TPT; ++k) {
            h[k] = hn[k];
            w[k] = wn[k];
        }
        __syncthreads();
    }
}

// Fused pass B: per W-column tile of one unit, column IFFT of each plane in
// the order DyDxz, DxDz, DxxDzz, DyxDyz, permute, fill epilogue.  The next
// plane (or the next tile's first plane) is prefetched into registers while
// the current one is transformed.  Values carried between planes (Dy/Dxz,
// then Dxx/Dzz) sit in LDS (lane-private slots) when they fit.
template <int N, int P>
__global__ __launch_bounds__(col_tile(N) * N / kElems) void k_pass_b2(DevView v, int items) {
    using CT = ColTile<N>;
    using E = typename CT::E;
    using TW = typename CT::TW;
    constexpr int W = CT::W;
    constexpr int T = CT::T;
    constexpr int RL = CT::RL;
    constexpr bool kKeepLds = (E::LDS_ELEMS + TW::kLdsEntries + kElems * T) * 8 <= 160 * 1024;
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    __shared__ float2 keep_lds[kKeepLds ? kElems * T : 1];
    TW::load(twl, v.tw, threadIdx.x, T);
    const float2* tws = TW::table(twl, v.tw);
    constexpr int order[4] = {1, 0, 3, 2};
    const int lb = CT::lane_b(), lj = CT::lane_j();
    const int voff8 = (lj * N + lb) * 8, voff16 = (lj * N + lb) * 16;

    float2 keep_reg[kKeepLds ? 1 : kElems];
    auto kput = [&](int i, float2 x) {
        if constexpr (kKeepLds) keep_lds[i * T + threadIdx.x] = x;
        else keep_reg[i] = x;
    };
    auto kget = [&](int i) -> float2 {
        if constexpr (kKeepLds) return keep_lds[i * T + threadIdx.x];
        else return keep_reg[i];
    };
    auto win8 = [&](const float2* base, int item) {
        const int u = item / CT::tiles, x0 = (item % CT::tiles) * W;
        return make_win(base + (size_t)u * N * N + x0, (unsigned)((N * N - x0) * 8));
    };
    auto win16 = [&](const float4* base, int item) {
        const int u = item / CT::tiles, x0 = (item % CT::tiles) * W;
        return make_win(base + (size_t)u * N * N + x0, (unsigned)((N * N - x0) * 16));
    };
    auto load = [&](int item, int p, float2 (&d)[kElems]) {
        const Win w = win8(v.plane[p], item);
#pragma unroll
        for (int i = 0; i < kElems; ++i) d[i] = bload2(w, voff8, CT::in_dy(i) * N * 8);
    };

    float2 cur[kElems], nxt[kElems];
    int item = blockIdx.x;
    if (item < items) load(item, order[0], cur);
    __syncthreads();
    for (; item < items; item += gridDim.x) {
        const int x0 = (item % CT::tiles) * W;
#pragma unroll
        for (int pi = 0; pi < P; ++pi) {
            const int p = order[pi];
            if (pi + 1 < P) load(item, order[pi + 1], nxt);
            else if (item + (int)gridDim.x < items) load(item + gridDim.x, order[0], nxt);
            float tb[kElems];
            if (p == 3) {
                const Win rt = win16(v.turb, item);
#pragma unroll
                for (int m = 0; m < kElems / RL; ++m)
#pragma unroll
                    for (int q = 0; q < RL; ++q) tb[m * RL + q] = bload1(rt, voff16, CT::out_dy(m, q) * N * 16);
            }
            const Win wd = win16(v.disp, item), wt = win16(v.turb, item), wv = win16(v.deriv, item);
            auto emit = [&](int m, int q, float2 val) {
                const int i = m * RL + q;
                const int dy = CT::out_dy(m, q);
                const float s = perm_sign(x0 + lb, lj + dy);
                const float re = val.x * s, im = val.y * s;
                const int so = dy * N * 16;
                if (p == 1) {  // DyDxz: keep Dy, Dxz
                    kput(i, make_float2(re, im));
                } else if (p == 0) {  // DxDz: DISP = (Dx, Dy, Dz, 1)
                    gstore4(make_float4(re, kget(i).x, im, 1.0f), wd, voff16, so);
                } else if (p == 3) {  // DxxDzz: foam (needs Dxz), then keep Dxx, Dzz
                    const float foam = foam_update(tb[i], re, im, kget(i).y);
                    gstore4(make_float4(foam, foam, foam, foam), wt, voff16, so);
                    kput(i, make_float2(re, im));
                } else {  // DyxDyz: DERIV = (Dyx, Dyz, Dxx, Dzz), NORMAL
                    const float2 k = kget(i);
                    gstore4(make_float4(re, im, k.x, k.y), wv, voff16, so);
                    if (v.normals) gstore4(normal_from_deriv(re, im, k.x, k.y), win16(v.normal, item), voff16, so);
                }
            };
            E::run_regs(cur, lds, tws, emit);
#pragma unroll
            for (int i = 0; i < kElems; ++i) cur[i] = nxt[i];
            __syncthreads();
        }
    }
}

// --------------------------------------------------------------- launch
int num_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}

template <class K>
int persistent_grid(K kernel, int threads, int items) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu <= 0)
        per_cu = 1;
    const int g = num_cus() * per_cu;
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
        hipLaunchKernelGGL((k_rows2<N, B>), dim3(g), dim3(T), 0, s, v->plane[p], total, v->tw);
        return hipGetLastError();
    }
    static hipError_t go(const DevView* v, int p, int np, hipStream_t s) {
        return go_b<rows_per_item(N)>(v, p, np, s);
    }
};
template <int N>
struct Cols2 {
    static hipError_t go(const DevView* v, int p, int np, hipStream_t s) {
        constexpr int W = cols2_w(N);
        constexpr int T = W * N / kElems;
        const int items = np * v->units * (N / W);
        const int g = persistent_grid(k_cols2<N>, T, items);
        hipLaunchKernelGGL(k_cols2<N>, dim3(g), dim3(T), 0, s, v->plane[p], items, v->tw);
        return hipGetLastError();
    }
};
template <int N>
struct PassA2 {
    template <int P>
    static hipError_t go_p(const DevView* v, float t, hipStream_t s) {
        constexpr int RB = pa_rows2<N, P>();
        constexpr int T = RB * P * N / kElems;
        const int total = v->units * N;
        const int items = (total + RB - 1) / RB;
        const int g = persistent_grid(k_pass_a2<N, P>, T, items);
        hipLaunchKernelGGL((k_pass_a2<N, P>), dim3(g), dim3(T), 0, s, *v, t, total);
        return hipGetLastError();
    }
    static hipError_t go(const DevView* v, float t, hipStream_t s) {
        return v->planes == 4 ? go_p<4>(v, t, s) : go_p<2>(v, t, s);
    }
};
template <int N>
struct PassB2 {
    template <int P>
    static hipError_t go_p(const DevView* v, hipStream_t s) {
        constexpr int W = col_tile(N);
        constexpr int T = W * N / kElems;
        const int items = v->units * (N / W);
        const int g = persistent_grid(k_pass_b2<N, P>, T, items);
        hipLaunchKernelGGL((k_pass_b2<N, P>), dim3(g), dim3(T), 0, s, *v, items);
        return hipGetLastError();
    }
    static hipError_t go(const DevView* v, hipStream_t s) { return v->planes == 4 ? go_p<4>(v, s) : go_p<2>(v, s); }
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
hipError_t launch_pass_a_v2(const DevView& v, float t, hipStream_t s) { return dispatch_n<PassA2>(v.n, &v, t, s); }
hipError_t launch_pass_b_v2(const DevView& v, hipStream_t s) { return dispatch_n<PassB2>(v.n, &v, s); }

}  // namespace ocean
