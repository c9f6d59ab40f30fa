// The fused frame: pass A (rows) and pass B (columns, N <= 1024) through a
// column-tile-major intermediate.
//
// Pass A3 (k_pass_a3, every N): evolve + row IFFT.  A workgroup owns RB rows and
//   all P planes of them.  The Stockham plan starts with radix R0 = 16/P so that
//   in stage 0 one lane holds every plane of R0 texels: the lane evolves those
//   texels (TimeDependentSpectrum.compute:20-47) and runs the first butterflies
//   on the results in registers -- no LDS round trip for the evolve.  The wave
//   data (kx, 1/|k|, kz, omega) is recomputed from (x, y, cascade) with the init
//   kernel's own arithmetic (spectrum_math.h wave_data, bit-identical) instead
//   of being read: 16 B/texel less HBM traffic.  Outputs go to the tile-major
//   intermediate [p][u][x/W][y][W], W = inter_w(N) (4 for small jobs at N <= 512,
//   ocean_create).
// Pass A4 (k_pass_a4, N = 512 / 1024 with 4 planes): the same per row pair
//   (y, N - y), sharing wave data and exp(i omega t) between k and -k and
//   reading h0 once through h0k (see the kernel).
// Pass B3 (k_pass_b3, N <= 1024): per W-column tile, column IFFT of each plane
//   from one contiguous 8*W*N-byte block, permute, fill/foam epilogue; the foam
//   state is a compact float in the same tile-major layout (4 B read + 4 B write
//   instead of a 16 B RGBA read), TURB is written as its broadcast image.
//   N >= 2048: fft4k.hip.
//
// Bytes per texel-cascade (P = 4): pass A 16 (h0; 8 for A4) + 32 (planes);
// pass B 32 (planes) + 4 + 4 (foam) + 48 (DISP, DERIV, TURB) = 88.
#include <type_traits>

#include "fft_engine.h"
#include "spectrum_math.h"

namespace ocean {
namespace {

constexpr int pa3_rows(int N, int RS = 2) { return N >= 1024 * RS ? 1 : 1024 * RS / N; }

// RS: row-sets per workgroup (RB = pa3_rows(N, RS) rows); PF: prefetch the
// next item's h0 before this item's transform (its loads are then ahead of
// this item's stores in the in-order vmcnt queue, so waiting for them never
// waits for the stores); BAND: a
// column band narrower than N (stores outside it skipped; a separate instance so
// that the whole-band frame pays no per-store test).  EPF (without PF): the next item's h0 is
// loaded into h as soon as the evolve has read it, in flight across the stages (+16-19 VGPRs:
// N = 4096 only, where the workgroup's occupancy does not change); else after the stages.
template <int N, int P, int RS, bool PF, bool BAND = false, int WT = 0, bool EPF = false>
__global__ __launch_bounds__(pa3_rows(N, RS) * P * N / kElems) void k_pass_a3(DevView v, float time, int total_rows) {
    constexpr int RB = pa3_rows(N, RS);
    constexpr int FIRST = 16 / P;
    using TW = StageTwLds<N, FIRST>;
    using E = Engine<N, RB * P, false, true, FIRST, TW>;
    constexpr int T = E::THREADS;
    constexpr int R0 = E::R0;             // = FIRST (texels per lane)
    constexpr int NJ = N / R0;            // stage-0 butterflies per sequence
    constexpr int W = WT ? WT : inter_w(N);  // WT: narrow tiles of a small job (ocean_create)
    constexpr int TILES = N / W;
    constexpr int NSL = N / E::RL;        // last-stage Ns
    static_assert(T / NJ == RB, "stage-0 mapping: lane -> (row, j), butterfly m -> plane m");
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    TW::load(twl, v.tw, threadIdx.x, T);
    const float2* tws = TW::table(twl, v.tw);
    // per-cascade band constants in LDS: a vector load here would be waited on
    // with vmcnt(0) together with the previous item's stores and the prefetch
    __shared__ WaveBand band[kMaxCascades];
    if ((int)threadIdx.x < v.C) band[threadIdx.x] = wave_band(v.casc + threadIdx.x * 5);
    const int rr = (int)threadIdx.x / NJ, j = (int)threadIdx.x % NJ;  // stage-0 lane coordinates
    const int items = (total_rows + RB - 1) / RB;

    float4 h[R0], hn[PF ? R0 : 1];
    auto load = [&](int item, float4* hh) {
        const int rows = min(RB, total_rows - item * RB);
        const Win w = make_win(v.h0 + (size_t)item * RB * N, (unsigned)(rows * N * 16));
#pragma unroll
        for (int r = 0; r < R0; ++r) hh[r] = bload4(w, (rr * N + j) * 16, r * NJ * 16);  // past-end rows read 0
    };
    // N >= 2048: deal consecutive rows to one XCD (blockIdx b runs on XCD b % 8).
    // Introduced for 4-wide tiles, whose 32-byte rows of 4 consecutive rows share a
    // 128-B line that one L2 then merges; today's 16-wide tile rows are whole lines
    int item = (N >= 2048 && gridDim.x % 8 == 0) ? (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)blockIdx.x / 8
                                                  : (int)blockIdx.x;
    if (item < items) load(item, h);
    __syncthreads();  // twiddles, band
    for (; item < items; item += gridDim.x) {
        const int next = item + gridDim.x;
        if constexpr (PF) {
            if (next < items) load(next, hn);
        }
        // stage-0 inputs: plane m of texel x = j + r*NJ of row (item*RB + rr)
        const int row = item * RB + rr;
        const int u = row / N, y = row % N;
        const WaveBand wb = band[(u + v.c0) % v.C];
        float2 in[kElems];
#pragma unroll
        for (int r = 0; r < R0; ++r) {
            const Planes4 o = evolve_texel(h[r], wave_data(j + r * NJ, y, N, wb, v.gravity), time);
#pragma unroll
            for (int m = 0; m < P; ++m) in[m * R0 + r] = o.p[m];
        }
        if constexpr (!PF && EPF) {
            if (next < items) load(next, h);
        }
        // outputs: sequence b = p*RB + rr', element x -> tplane[p][u'][x/W][y'][x%W]
        auto emit = [&](int m, int q, float2 val) {
            int b, jj;
            E::template bj<E::RL>((int)threadIdx.x + m * T, b, jj);
            const int p = b / RB, r2 = b % RB;
            const int row2 = item * RB + r2;
            // column band: rows are transformed whole, only the band's columns stored
            if (row2 < total_rows && (!BAND || (unsigned)(jj + q * NSL - v.x0) < (unsigned)v.nx)) {
                const int u2 = row2 / N, y2 = row2 % N;
                float2* rowp = v.tplane + (size_t)p * v.inter_stride + ((size_t)u2 * TILES * N + y2) * W;
                if constexpr (NSL % W == 0) {
                    // x = jj + q*NSL: x/W = jj/W + q*NSL/W, x%W = jj%W (compile-time tile stride)
                    float2* dst = rowp + (size_t)(jj / W) * N * W + (jj % W);
                    dst[(size_t)q * (NSL / W) * N * W] = val;
                } else {
                    const int x = jj + q * NSL;
                    rowp[(size_t)(x / W) * N * W + (x % W)] = val;
                }
            }
        };
        E::run_regs(in, lds, tws, emit);
        if constexpr (PF) {
#pragma unroll
            for (int r = 0; r < R0; ++r) h[r] = hn[r];
        }
        __syncthreads();
        if constexpr (!PF && !EPF) {
            if (next < items) load(next, h);
        }
    }
}

// Pass B: one item = (unit, W-column tile); planes in the order DyDxz, DxDz,
// DxxDzz, DyxDyz with the next PFD planes prefetched into registers.
template <int N, int P, int PFD = 1, int WT = 0>
__global__ __launch_bounds__((WT ? WT : b3_w(N)) * N / kElems) void k_pass_b3(DevView v, int items) {
    using CT = ColTile<N, WT ? WT : b3_w(N)>;
    using E = typename CT::E;
    using TW = typename CT::TW;
    constexpr int W = CT::W;
    constexpr int T = CT::T;
    constexpr int RL = CT::RL;
    constexpr int TILE = W * N;
    constexpr bool kKeepLds = (E::LDS_ELEMS + TW::kLdsEntries + kElems * T) * 8 <= 160 * 1024;
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    __shared__ float2 keep_lds[kKeepLds ? kElems * T : 1];
    TW::load(twl, v.tw, threadIdx.x, T);
    const float2* tws = TW::table(twl, v.tw);
    constexpr int order[4] = {1, 0, 3, 2};
    const int lb = CT::lane_b(), lj = CT::lane_j();
    const int toff = lj * W + lb;                 // lane's element in a tile block
    const int voff16 = (lj * N + lb) * 16;        // lane's texel in a [y][x] float4 texture window

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
    auto full = [&](int item) { return (item / bnt) * CT::tiles + bt0 + item % bnt; };
    auto win16 = [&](const float4* base, int ft) {
        const int u = ft / CT::tiles, x0 = (ft % CT::tiles) * W;
        return make_win(base + (size_t)u * N * N + x0, (unsigned)((N * N - x0) * 16));
    };
    auto load = [&](int item, int p, float2 (&d)[kElems]) {
        const Win w = make_win(v.tplane + (size_t)p * v.inter_stride + (size_t)full(item) * TILE, TILE * 8);
#pragma unroll
        for (int i = 0; i < kElems; ++i) d[i] = bload2(w, toff * 8, CT::in_dy(i) * W * 8);
    };

    // PFD planes in flight ahead of the one being transformed (register ring)
    // (PFD = 0: no prefetch, each plane loaded when its step starts -- N = 4096,
    // where 1024 lanes leave 128 VGPRs)
    float2 cur[kElems], nxt[PFD > 0 ? kElems : 1], nx2[PFD > 1 ? kElems : 1];
    int item = blockIdx.x;
    if (item < items && PFD > 0) {
        load(item, order[0], cur);
        if constexpr (PFD > 1) load(item, order[1], nxt);
    }
    __syncthreads();
    for (; item < items; item += gridDim.x) {
        const int ft = full(item);
        const int x0 = (ft % CT::tiles) * W;
        float* foam = v.foam + (size_t)ft * TILE + toff;
        float fb[kElems];
#pragma unroll
        for (int pi = 0; pi < P; ++pi) {
            const int p = order[pi];
            // foam state for the DxxDzz plane: loaded one plane ahead and before that
            // step's tile prefetch, so waiting for it never waits for the prefetch
            if (pi + 1 < P && order[pi + 1] == 3) {
                const Win rf = make_win(v.foam + (size_t)ft * TILE, TILE * 4);
#pragma unroll
                for (int m = 0; m < kElems / RL; ++m)
#pragma unroll
                    for (int q = 0; q < RL; ++q) fb[m * RL + q] = bload1(rf, toff * 4, CT::out_dy(m, q) * W * 4);
            }
            if constexpr (PFD == 0) {
                load(item, p, cur);
            } else if constexpr (PFD > 1) {
                if (pi + 2 < P) load(item, order[pi + 2], nx2);
                else if (item + (int)gridDim.x < items) load(item + gridDim.x, order[pi + 2 - P], nx2);
            } else {
                if (pi + 1 < P) load(item, order[pi + 1], nxt);
                else if (item + (int)gridDim.x < items) load(item + gridDim.x, order[0], nxt);
            }
            const Win wd = win16(v.disp, ft), wt = win16(v.turb, ft), wv = win16(v.deriv, ft);
            // texture outputs are streamed (nontemporal): nothing in the frame reads them
            // back, and default-policy stores would evict h0k, the intermediate and the
            // foam state from the Infinity Cache before the next frame re-reads them
            auto st4 = [&](float4 x, const Win& w, int voff, int soff) { gstore4_nt(x, w, voff, soff); };
            auto stf = [&](float* a, float x) { *a = x; };
            auto emit = [&](int m, int q, float2 val) {
                const int i = m * RL + q;
                const int dy = CT::out_dy(m, q);
                const float s = perm_sign(x0 + lb, lj + dy);
                const float re = val.x * s, im = val.y * s;
                const int so = dy * N * 16;
                if (p == 1) {  // DyDxz: keep Dy, Dxz
                    kput(i, make_float2(re, im));
                } else if (p == 0) {  // DxDz: DISP = (Dx, Dy, Dz, 1)
                    st4(make_float4(re, kget(i).x, im, 1.0f), wd, voff16, so);
                } else if (p == 3) {  // DxxDzz: foam (needs Dxz), then keep Dxx, Dzz
                    const float f = foam_update(fb[i], re, im, kget(i).y);
                    stf(&foam[dy * W], f);
                    st4(make_float4(f, f, f, f), wt, voff16, so);
                    kput(i, make_float2(re, im));
                } else {  // DyxDyz: DERIV = (Dyx, Dyz, Dxx, Dzz), NORMAL
                    const float2 k = kget(i);
                    st4(make_float4(re, im, k.x, k.y), wv, voff16, so);
                    if (v.normals) st4(normal_from_deriv(re, im, k.x, k.y), win16(v.normal, ft), voff16, so);
                }
            };
            E::run_regs(cur, lds, tws, emit);
#pragma unroll
            for (int i = 0; i < kElems; ++i) {
                if constexpr (PFD > 0) cur[i] = nxt[i];
                if constexpr (PFD > 1) nxt[i] = nx2[i];
            }
            __syncthreads();
        }
    }
}

// Pass B of a displacement-only frame (P = 2) with both planes at once: the workgroup's two halves
// (T lanes each) run the column transforms of DyDxz and DxDz side by side, each on its own LDS image
// (Engine SUB: lane = threadIdx.x % T; the halves meet at the same barriers), so an item is one
// transform's latency chain instead of two; the halves then swap Dy through LDS and the DxDz half
// stores DISP.  Small jobs (cfg2: one 512^2 cascade, one item per workgroup) are such chains.
template <int N, int WT = 0>
__global__ __launch_bounds__(2 * (WT ? WT : b3_w(N)) * N / kElems) void k_pass_b2d(DevView v, int items) {
    using CT = ColTile<N, WT ? WT : b3_w(N)>;
    using TW = typename CT::TW;
    constexpr int W = CT::W;
    using E = Engine<N, W, true, (CT::E::LDS_ELEMS != N * W), 16, TW, kElems, true>;
    static_assert(E::LDS_ELEMS == CT::E::LDS_ELEMS, "same layout as the column-tile engine");
    constexpr int T = CT::T;
    constexpr int RL = CT::RL;
    constexpr int TILE = W * N;
    __shared__ float2 lds[2][E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    __shared__ float keepy[kElems * T];
    TW::load(twl, v.tw, threadIdx.x, 2 * T);
    const float2* tws = TW::table(twl, v.tw);
    const int half = (int)threadIdx.x / T;  // 0: DyDxz (plane 1), 1: DxDz (plane 0); whole waves
    const int t = (int)threadIdx.x % T;
    const int lb = t % W, lj = t / W;
    const int toff = lj * W + lb;
    const int voff16 = (lj * N + lb) * 16;
    const int plane = half ? 0 : 1;
    const int bt0 = v.x0 / W, bnt = v.nx / W;
    auto full = [&](int item) { return (item / bnt) * CT::tiles + bt0 + item % bnt; };
    auto load = [&](int item, float2 (&d)[kElems]) {
        const Win w = make_win(v.tplane + (size_t)plane * v.inter_stride + (size_t)full(item) * TILE, TILE * 8);
#pragma unroll
        for (int i = 0; i < kElems; ++i) d[i] = bload2(w, toff * 8, CT::in_dy(i) * W * 8);
    };
    float2 cur[kElems], nxt[kElems], kxz[kElems];
    int item = blockIdx.x;
    if (item < items) load(item, cur);
    __syncthreads();
    for (; item < items; item += gridDim.x) {
        if (item + (int)gridDim.x < items) load(item + gridDim.x, nxt);
        const int ft = full(item);
        const int u = ft / CT::tiles, x0 = (ft % CT::tiles) * W;
        auto emit = [&](int m, int q, float2 val) {
            const int i = m * RL + q;
            const float s = perm_sign(x0 + lb, lj + CT::out_dy(m, q));
            if (half == 0) keepy[i * T + t] = val.x * s;          // Dy
            else kxz[i] = make_float2(val.x * s, val.y * s);      // Dx, Dz
        };
        E::run_regs(cur, lds[half], tws, emit);
        __syncthreads();
        if (half == 1) {  // DISP = (Dx, Dy, Dz, 1), streamed
            const Win wd = make_win(v.disp + (size_t)u * N * N + x0, (unsigned)((N * N - x0) * 16));
#pragma unroll
            for (int m = 0; m < kElems / RL; ++m)
#pragma unroll
                for (int q = 0; q < RL; ++q) {
                    const int i = m * RL + q;
                    gstore4_nt(make_float4(kxz[i].x, keepy[i * T + t], kxz[i].y, 1.0f), wd, voff16,
                               CT::out_dy(m, q) * N * 16);
                }
        }
#pragma unroll
        for (int i = 0; i < kElems; ++i) cur[i] = nxt[i];
        __syncthreads();
    }
}

// Pass B8 (N = 512, W = 4 narrow tiles, displacement only; cfg2): k_pass_b2d's two planes side by
// side with 8 values per lane instead of 16.  Each half (N W / 8 lanes, lane = column lb, butterfly
// lj) runs radix 8 in registers on rows lj + 64 r, then radix 8, 8 through LDS ([y][W] layout, one
// W-row of padding every 16 rows), twiddles from the base table exp(2 pi i m / N); the halves swap
// Dy through LDS and the DxDz half stores DISP.  Twice the lanes per item, half the per-lane chain.
template <int N, int W>
__global__ __launch_bounds__(2 * W * N / 8) void k_pass_b8(DevView v, int items) {
    static_assert(N == 512, "plan 8 x 8 x 8");
    constexpr int T = W * N / 8;  // lanes per half
    constexpr int NR = N / 8;     // butterflies per column and stage
    constexpr int TILE = W * N;
    constexpr int TILES = N / W;
    constexpr int IMG = TILE + (TILE / (16 * W)) * W;
    __shared__ float2 lds[2][IMG];
    __shared__ float2 twb[N];
    __shared__ float keepy[8 * T];
    for (int i = threadIdx.x; i < N; i += 2 * T) twb[i] = v.tw[i];
    const int half = (int)threadIdx.x / T;  // 0: DyDxz (plane 1), 1: DxDz (plane 0); whole waves
    const int t = (int)threadIdx.x % T;
    const int lb = t % W, lj = t / W;
    const int plane = half ? 0 : 1;
    float2* img = lds[half];
    auto li = [](int y, int b) { const int i = y * W + b; return i + (i / (16 * W)) * W; };
    const int bt0 = v.x0 / W, bnt = v.nx / W;
    auto full = [&](int item) { return (item / bnt) * TILES + bt0 + item % bnt; };
    auto load = [&](int item, float2 (&d)[8]) {
        const Win w = make_win(v.tplane + (size_t)plane * v.inter_stride + (size_t)full(item) * TILE, TILE * 8);
#pragma unroll
        for (int r = 0; r < 8; ++r) d[r] = bload2(w, (lj * W + lb) * 8, r * NR * W * 8);
    };
    // Stockham stage (NS, 8) of butterfly lj of column lb from LDS
    auto stage = [&](auto ns_c, float2 (&x)[8]) {
        constexpr int NS = decltype(ns_c)::value;
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = img[li(lj + r * NR, lb)];
        __syncthreads();
        const int k = lj & (NS - 1);
#pragma unroll
        for (int r = 1; r < 8; ++r) x[r] = cmul(x[r], twb[r * k * (N / (NS * 8))]);
        Idft<8>::run(x);
    };
    float2 cur[8], nxt[8], kxz[8];
    int item = blockIdx.x;
    if (item < items) load(item, cur);
    __syncthreads();  // twiddles
    for (; item < items; item += gridDim.x) {
        if (item + (int)gridDim.x < items) load(item + gridDim.x, nxt);
        const int ft = full(item);
        const int u = ft / TILES, x0 = (ft % TILES) * W;
        // stage 0 (NS = 1): outputs y = 8 lj + q
        Idft<8>::run(cur);
#pragma unroll
        for (int q = 0; q < 8; ++q) img[li(8 * lj + q, lb)] = cur[q];
        __syncthreads();
        float2 x[8];
        stage(std::integral_constant<int, 8>{}, x);
        {
            const int y0 = (lj / 8) * 64 + (lj & 7);
#pragma unroll
            for (int q = 0; q < 8; ++q) img[li(y0 + q * 8, lb)] = x[q];
        }
        __syncthreads();
        stage(std::integral_constant<int, 64>{}, x);  // last: outputs y = lj + 64 q
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float s = perm_sign(x0 + lb, lj + q * NR);
            if (half == 0) keepy[q * T + t] = x[q].x * s;         // Dy
            else kxz[q] = make_float2(x[q].x * s, x[q].y * s);   // Dx, Dz
        }
        __syncthreads();
        if (half == 1) {  // DISP = (Dx, Dy, Dz, 1), streamed
            const Win wd = make_win(v.disp + (size_t)u * N * N + x0, (unsigned)((N * N - x0) * 16));
#pragma unroll
            for (int q = 0; q < 8; ++q)
                gstore4_nt(make_float4(kxz[q].x, keepy[q * T + t], kxz[q].y, 1.0f), wd, (lj * N + lb) * 16,
                           q * NR * N * 16);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) cur[r] = nxt[r];
        __syncthreads();
    }
}

// Pass A over mirror pairs (N = 1024, P = 4; docs/MEASUREMENTS.md section 3, "pass A4").  Item i of
// unit u covers rows y1 = i and y2 = N - i for 0 < i < N/2; item 0 covers rows
// 0 and N/2, which are their own mirrors and are evolved texel by texel.  The
// texel k = (x, y1) and its mirror -k = ((N - x) % N, y2) have the same |k|,
// hence the same wave data up to the signs of kx, kz and the same phase factor
// exp(i omega t); their h0 halves are each other's conjugates
// (InitialSpectrum.compute:135-143), so the pair needs h0k at two texels (16 B)
// instead of h0 at two texels (32 B) and one wave_data + sincos instead of two.
// Lane j (N/4 lanes) holds stage-0 butterfly j of row y1 and butterfly
// jm = (NJ - j) % NJ of row y2, whose texels are the mirrors of its own: two
// radix-4 butterflies x 4 planes = 32 values per lane (Engine EL = 32).
//
// PH = 2 planes per LDS pass: 4 of the 8 sequences in LDS (planes p0, p0 + 1 of both rows),
// the stages run twice per item: 43.5 KiB of LDS instead of 78 KiB, so 3 workgroups share a
// CU instead of 2 and the per-workgroup latency chain (evolve -> LDS stages -> stores)
// overlaps better: 38.6 -> 33.0 us at cfg3 (docs/MEASUREMENTS.md).
//
// P = 2 (displacement-only frames, N = 256): both planes in one LDS pass.
template <int N, bool BAND = false, int WT = 0, int P = 4>
__global__ __launch_bounds__(N / 4) void k_pass_a4(DevView v, float time, int items_per_unit, int items) {
    constexpr int R0 = 4, RB = 2, EL = 2 * P * R0, PH = 2;
    using TW = StageTw<N, R0>;
    using E = Engine<N, RB * PH, false, true, R0, TW, EL * PH / P>;
    constexpr int T = E::THREADS;
    constexpr int NJ = N / R0;
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
        u = it / items_per_unit;
        const int i = it - u * items_per_unit;
        y1 = i;
        y2 = i ? N - i : N / 2;
    };
    // h0k at texel x_r = j + r NJ of row y1 and at its mirror (N - x_r) % N of row y2
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
    float2 A[R0], B[R0], An[R0], Bn[R0];
    int item = blockIdx.x;
    if (item < items) load_pair(item, A, B);
    __syncthreads();  // twiddles, band
    for (; item < items; item += gridDim.x) {
        const int next = item + gridDim.x;
        if (next < items) load_pair(next, An, Bn);
        int u, y1, y2;
        rows_of(item, u, y1, y2);
        const WaveBand wb = band[(u + v.c0) % v.C];
        float2 in[EL];  // slot (s*4 + p)*4 + r: set s (row y1 / y2), plane p, stage-0 input r
        if (y1 != 0) {
            float2 mir[P][R0];  // set-2 values in mirror order (slot r = mirror of set-1 slot r)
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                const int x = j + r * NJ;
                const float4 wd = wave_data(x, y1, N, wb, v.gravity);
                const Phase e = evolve_phase(wd.w, time);
                const Planes4 o = evolve_with(make_float4(A[r].x, A[r].y, B[r].x, -B[r].y), wd, e);
                // mirror: kx -> -kx (except the Nyquist column x = 0), kz -> -kz, same 1/|k| and omega
                const float4 wm = make_float4((j0 && r == 0) ? wd.x : -wd.x, wd.y, -wd.z, wd.w);
                const Planes4 om = evolve_with(make_float4(B[r].x, B[r].y, A[r].x, -A[r].y), wm, e);
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    in[p * R0 + r] = o.p[p];
                    mir[p][r] = om.p[p];
                }
            }
            // FFT slot r' of butterfly jm holds texel jm + r' NJ = mirror of slot r with
            // r' = R0 - 1 - r, or (R0 - r) % R0 on lane 0 (jm = 0)
#pragma unroll
            for (int p = 0; p < P; ++p)
#pragma unroll
                for (int r2 = 0; r2 < R0; ++r2) {
                    const float2 a = mir[p][R0 - 1 - r2], b = mir[p][(R0 - r2) & (R0 - 1)];
                    in[(P + p) * R0 + r2] = j0 ? b : a;
                }
        } else {
            // rows 0 and N/2: texels pair inside their row; no sharing (1 item in N/2)
            float2 am[R0], c[R0];
            const float2* r1 = v.h0k + ((size_t)u * N + y1) * N;
            const float2* r2 = v.h0k + ((size_t)u * N + y2) * N;
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                am[r] = r1[(N - j - r * NJ) & (N - 1)];
                c[r] = r2[j + r * NJ];
            }
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                const int x = j + r * NJ;
                const Planes4 o1 = evolve_texel(make_float4(A[r].x, A[r].y, am[r].x, -am[r].y),
                                                wave_data(x, y1, N, wb, v.gravity), time);
                const Planes4 o2 = evolve_texel(make_float4(c[r].x, c[r].y, B[r].x, -B[r].y),
                                                wave_data(x, y2, N, wb, v.gravity), time);
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    in[p * R0 + r] = o1.p[p];
                    in[(P + p) * R0 + r] = o2.p[p];
                }
            }
        }
        // stage 0 (radix 4) in registers; LDS sequence b = (p - p0) * 2 + s
        const int jb1 = (y1 != 0) ? jm : j;
#pragma unroll
        for (int g = 0; g < 2 * P; ++g) Idft<R0>::run(&in[g * R0]);
#pragma unroll
        for (int p0 = 0; p0 < P; p0 += PH) {
#pragma unroll
            for (int g = 0; g < 2 * P; ++g) {
                const int s = g / P, p = g % P;
                if (p < p0 || p >= p0 + PH) continue;
                float2* dst = lds + E::lidx((p - p0) * RB + s, (s ? jb1 : j) * R0);
#pragma unroll
                for (int q = 0; q < R0; ++q) dst[E::loff(q, 1)] = in[g * R0 + q];
            }
            __syncthreads();
            auto emit = [&](int m, int q, float2 val) {
                int b, jj;
                E::template bj<E::RL>((int)threadIdx.x + m * T, b, jj);
                if (BAND && (unsigned)(jj + q * NSL - v.x0) >= (unsigned)v.nx) return;  // outside the column band
                const int p = p0 + b / RB, y = (b % RB) ? y2 : y1;
                float2* dst = v.tplane + (size_t)p * v.inter_stride + ((size_t)u * TILES * N + y) * W +
                              (size_t)(jj / W) * N * W + (jj % W);
                dst[(size_t)q * (NSL / W) * N * W] = val;
            };
            E::template stages_from<1>(lds, tws, emit);
            __syncthreads();
        }
#pragma unroll
        for (int r = 0; r < R0; ++r) {
            A[r] = An[r];
            B[r] = Bn[r];
        }
    }
}

// Pass A8 (N = 512, two planes: small displacement-only jobs, cfg2; docs/MEASUREMENTS.md section 6): the
// mirror pairs of k_pass_a4 on N/2 lanes with 8 values each.  Lane j holds texels x = j, j + N/2
// of row y1 and their mirrors in row y2 (butterfly jm = (N/2 - j) % (N/2)), so it evolves two
// texel pairs instead of four; the row transform runs radix 2 in registers, then radix 8, 8
// (wave-private: wave w = sequence w) and 4 through LDS, twiddles from the base table
// exp(2 pi i m / N).  An item then has 4 waves instead of 2 and half the per-lane chain.
template <int N, int WT = 0>
__global__ __launch_bounds__(N / 2) void k_pass_a8(DevView v, float time, int items_per_unit, int items) {
    static_assert(N == 512, "plan 2 x 8 x 8 x 4");
    constexpr int T = N / 2, NB = 4;  // LDS sequence b = p * 2 + s (plane p, row set s)
    constexpr int W = WT ? WT : inter_w(N);
    constexpr int TILES = N / W;
    __shared__ float2 lds[padded(NB * N)];
    __shared__ float2 twb[N];
    __shared__ WaveBand band[kMaxCascades];
    for (int i = threadIdx.x; i < N; i += T) twb[i] = v.tw[i];
    if ((int)threadIdx.x < v.C) band[threadIdx.x] = wave_band(v.casc + threadIdx.x * 5);
    const int j = (int)threadIdx.x;
    const bool j0 = (j == 0);
    const int jm = (T - j) & (T - 1);
    const bool banded = v.nx != N;
    auto rows_of = [&](int it, int& u, int& y1, int& y2) {
        u = it / items_per_unit;
        const int i = it - u * items_per_unit;
        y1 = i;
        y2 = i ? N - i : N / 2;
    };
    float2 A[2], B[2];
    auto load_pair = [&](int it) {
        int u, y1, y2;
        rows_of(it, u, y1, y2);
        const float2* r1 = v.h0k + ((size_t)u * N + y1) * N;
        const float2* r2 = v.h0k + ((size_t)u * N + y2) * N;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            A[r] = r1[j + r * T];
            B[r] = r2[(N - j - r * T) & (N - 1)];
        }
    };
    // one Stockham stage (NS, R) over the four sequences from LDS; LAST hands (b, x, value) to emit
    auto stage = [&](auto ns_c, auto r_c, auto last_c, auto&& emit) {
        constexpr int NS = decltype(ns_c)::value, R = decltype(r_c)::value;
        constexpr bool LAST = decltype(last_c)::value;
        constexpr int NR = N / R, BF = NB * NR / T;
        float2 x[BF][R];
#pragma unroll
        for (int m = 0; m < BF; ++m) {
            const int g = j + m * T, b = g / NR, jj = g % NR;
#pragma unroll
            for (int r = 0; r < R; ++r) x[m][r] = lds[pad(b * N + jj + r * NR)];
        }
        if constexpr (NB * NR / T == 1 && NR == 64) __asm__ volatile("" ::: "memory");  // wave-private
        else __syncthreads();
#pragma unroll
        for (int m = 0; m < BF; ++m) {
            const int g = j + m * T, b = g / NR, jj = g % NR;
            const int k = jj & (NS - 1);
#pragma unroll
            for (int r = 1; r < R; ++r) x[m][r] = cmul(x[m][r], twb[r * k * (N / (NS * R))]);
            Idft<R>::run(x[m]);
            if constexpr (LAST) {
#pragma unroll
                for (int q = 0; q < R; ++q) emit(b, jj + q * NS, x[m][q]);
            } else {
                const int y0 = (jj / NS) * NS * R + k;
#pragma unroll
                for (int q = 0; q < R; ++q) lds[pad(b * N + y0 + q * NS)] = x[m][q];
            }
        }
    };
    using std::integral_constant;
    int item = blockIdx.x;
    if (item < items) load_pair(item);
    __syncthreads();  // twiddles, band
    for (; item < items; item += gridDim.x) {
        const int next = item + gridDim.x;
        int u, y1, y2;
        rows_of(item, u, y1, y2);
        const WaveBand wb = band[(u + v.c0) % v.C];
        float2 in[2][2][2];  // [row set s][plane p][texel slot r]
        if (y1 != 0) {
            float2 mir[2][2];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int x = j + r * T;
                const float4 wd = wave_data(x, y1, N, wb, v.gravity);
                const Phase e = evolve_phase(wd.w, time);
                const Planes4 o = evolve_with(make_float4(A[r].x, A[r].y, B[r].x, -B[r].y), wd, e);
                // mirror: kx -> -kx (except the Nyquist column x = 0), kz -> -kz, same 1/|k| and omega
                const float4 wm = make_float4((j0 && r == 0) ? wd.x : -wd.x, wd.y, -wd.z, wd.w);
                const Planes4 om = evolve_with(make_float4(B[r].x, B[r].y, A[r].x, -A[r].y), wm, e);
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    in[0][p][r] = o.p[p];
                    mir[p][r] = om.p[p];
                }
            }
            // the mirror of texel j + T r is texel (N - j - T r) % N: slot 1 - r of butterfly jm
            // (j != 0), slot r of butterfly 0 (j = 0)
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                in[1][p][0] = j0 ? mir[p][0] : mir[p][1];
                in[1][p][1] = j0 ? mir[p][1] : mir[p][0];
            }
        } else {
            // rows 0 and N/2: texels pair inside their row (1 item in N/2)
            const float2* r1 = v.h0k + ((size_t)u * N + y1) * N;
            const float2* r2 = v.h0k + ((size_t)u * N + y2) * N;
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int x = j + r * T;
                const float2 am = r1[(N - x) & (N - 1)], c = r2[x];
                const Planes4 o1 = evolve_texel(make_float4(A[r].x, A[r].y, am.x, -am.y),
                                                wave_data(x, y1, N, wb, v.gravity), time);
                const Planes4 o2 = evolve_texel(make_float4(c.x, c.y, B[r].x, -B[r].y),
                                                wave_data(x, y2, N, wb, v.gravity), time);
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    in[0][p][r] = o1.p[p];
                    in[1][p][r] = o2.p[p];
                }
            }
        }
        if (next < items) load_pair(next);  // in flight across the stages
        // stage 0 (radix 2, NS = 1) in registers: outputs y = 2 jb + q
        const int jb1 = (y1 != 0) ? jm : j;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                Idft<2>::run(in[s][p]);
                const int b = p * 2 + s, jb = s ? jb1 : j;
                lds[pad(b * N + 2 * jb)] = in[s][p][0];
                lds[pad(b * N + 2 * jb + 1)] = in[s][p][1];
            }
        __syncthreads();
        auto none = [](int, int, float2) {};
        stage(integral_constant<int, 2>{}, integral_constant<int, 8>{}, std::false_type{}, none);
        stage(integral_constant<int, 16>{}, integral_constant<int, 8>{}, std::false_type{}, none);
        __syncthreads();
        auto emit = [&](int b, int x, float2 val) {
            if (banded && (unsigned)(x - v.x0) >= (unsigned)v.nx) return;  // outside the column band
            const int p = b >> 1, y = (b & 1) ? y2 : y1;
            float2* dst = v.tplane + (size_t)p * v.inter_stride + ((size_t)u * TILES * N + y) * W +
                          (size_t)(x / W) * N * W + (x % W);
            *dst = val;
        };
        stage(integral_constant<int, 128>{}, integral_constant<int, 4>{}, std::true_type{}, emit);
        __syncthreads();  // LDS reused by the next item
    }
}

template <class K>
int grid3(K kernel, int threads, int items) {
    const int g = device_cus() * resident_per_cu((const void*)kernel, threads);
    return items < g ? items : g;
}

// EPF at N = 4096: the next row's h0 in flight across the stages (641 against 658 us, docs/MEASUREMENTS.md)
template <int N, int P, int RS, bool PF, bool BAND = false, int WT = 0>
hipError_t go_a3k(const DevView& v, float t, hipStream_t s) {
    if constexpr (WT == 0 && N >= 128 && N <= 1024) {
        if (v.tile_w != inter_w(N)) return go_a3k<N, P, RS, PF, BAND, 4>(v, t, s);
    }
    if constexpr (!BAND) {
        if (v.nx != N) return go_a3k<N, P, RS, PF, true, WT>(v, t, s);
    }
    constexpr int RB = pa3_rows(N, RS);
    constexpr int T = RB * P * N / kElems;
    const int total = v.units * N;
    const int items = (total + RB - 1) / RB;
    constexpr bool EPF = (N == 4096);
    const int g = grid3(k_pass_a3<N, P, RS, PF, BAND, WT, EPF>, T, items);
    launch((k_pass_a3<N, P, RS, PF, BAND, WT, EPF>), dim3(g), dim3(T), 0, s, v, t, total);
    return hipGetLastError();
}

// N = 1024, 4 planes: 2 rows per workgroup (512 lanes) with the next item's h0
// prefetched; other sizes: pa3_rows(N, 1) rows.
template <int N, int P>
hipError_t go_a3(const DevView& v, float t, hipStream_t s) {
    if constexpr (N == 1024 && P == 4) return go_a3k<N, P, 2, true>(v, t, s);
    return go_a3k<N, P, 1, false>(v, t, s);
}

template <int N, int P, int PFD, int WT = 0>
hipError_t go_b3k(const DevView& v, hipStream_t s) {
    if constexpr (WT == 0 && N >= 128 && N <= 1024) {
        if (v.tile_w != inter_w(N)) return go_b3k<N, P, PFD, 4>(v, s);
    }
    constexpr int W = WT ? WT : b3_w(N);
    constexpr int T = W * N / kElems;
    const int items = v.units * (v.nx / W);
    const int g = grid3(k_pass_b3<N, P, PFD, WT>, T, items);
    launch((k_pass_b3<N, P, PFD, WT>), dim3(g), dim3(T), 0, s, v, items);
    return hipGetLastError();
}

// narrow (4-column) tiles only: two images of a wide tile exceed the CU's LDS
template <int N>
hipError_t go_b2d(const DevView& v, hipStream_t s) {
    constexpr int W = 4;
    constexpr int T = 2 * W * N / kElems;
    const int items = v.units * (v.nx / W);
    const int g = grid3(k_pass_b2d<N, W>, T, items);
    launch((k_pass_b2d<N, W>), dim3(g), dim3(T), 0, s, v, items);
    return hipGetLastError();
}

template <int N>
hipError_t go_b8(const DevView& v, hipStream_t s) {
    constexpr int W = 4;
    constexpr int T = 2 * W * N / 8;
    const int items = v.units * (v.nx / W);
    const int g = grid3(k_pass_b8<N, W>, T, items);
    launch((k_pass_b8<N, W>), dim3(g), dim3(T), 0, s, v, items);
    return hipGetLastError();
}

// Two planes in flight at N = 1024 (one workgroup per CU, registers to spare).  Displacement-only
// frames (P = 2) on narrow tiles run both planes side by side: pass B8 at N = 512 (8 values per
// lane), k_pass_b2d at N = 128..256.
template <int N, int P>
hipError_t go_b3(const DevView& v, hipStream_t s) {
    if constexpr (P == 2 && N == 512) {
        if (v.tile_w == 4) return go_b8<N>(v, s);
    }
    if constexpr (P == 2 && N >= 128 && N <= 256) {
        if (v.tile_w == 4) return go_b2d<N>(v, s);
    }
    if constexpr (N == 1024) return go_b3k<N, P, 2>(v, s);
    return go_b3k<N, P, 1>(v, s);
}

template <int N, bool BAND = false, int WT = 0, int P = 4>
hipError_t go_a4(const DevView& v, float t, hipStream_t s) {
    if constexpr (WT == 0) {
        if (v.tile_w != inter_w(N)) return go_a4<N, BAND, 4, P>(v, t, s);
    }
    if constexpr (!BAND) {
        if (v.nx != N) return go_a4<N, true, WT, P>(v, t, s);
    }
    constexpr int T = N / 4;
    const int ipu = N / 2;
    const int items = v.units * ipu;
    const int g = grid3(k_pass_a4<N, BAND, WT, P>, T, items);
    launch((k_pass_a4<N, BAND, WT, P>), dim3(g), dim3(T), 0, s, v, t, ipu, items);
    return hipGetLastError();
}

template <int N, int WT>
hipError_t go_a8(const DevView& v, float t, hipStream_t s) {
    constexpr int T = N / 2;
    const int ipu = N / 2;
    const int items = v.units * ipu;
    const int g = grid3(k_pass_a8<N, WT>, T, items);
    launch((k_pass_a8<N, WT>), dim3(g), dim3(T), 0, s, v, t, ipu, items);
    return hipGetLastError();
}

}  // namespace

// N = 512 / 1024 with four planes; N = 256 / 512 displacement-only (two planes)
bool pass_a4_supported(int n, int planes) {
    if (planes == 2) return n == 256 || n == 512;
    return planes == 4 && (n == 512 || n == 1024);
}

// P = 2 at N = 512: pass A8 (256 lanes, 8 values each; 6.64 against 7.47 us for pass A4's two-plane
// layout at cfg2, docs/MEASUREMENTS.md section 6)
hipError_t launch_pass_a_v4(const DevView& v, float t, hipStream_t s) {
    if (!pass_a4_supported(v.n, v.planes) || !v.h0k) return hipErrorInvalidValue;
    if (v.planes == 2) {
        if (v.n == 256) return go_a4<256, false, 0, 2>(v, t, s);
        return v.tile_w == inter_w(512) ? go_a8<512, 0>(v, t, s) : go_a8<512, 4>(v, t, s);
    }
    return v.n == 512 ? go_a4<512>(v, t, s) : go_a4<1024>(v, t, s);
}

hipError_t launch_pass_a_v3(const DevView& v, float t, hipStream_t s) {
#define OCEAN_A3(NN)                                                                 \
    case NN:                                                                         \
        return v.planes == 4 ? go_a3<NN, 4>(v, t, s) : go_a3<NN, 2>(v, t, s);
    switch (v.n) {
        OCEAN_A3(16)
        OCEAN_A3(32)
        OCEAN_A3(64)
        OCEAN_A3(128)
        OCEAN_A3(256)
        OCEAN_A3(512)
        OCEAN_A3(1024)
        OCEAN_A3(2048)
        OCEAN_A3(4096)
    }
#undef OCEAN_A3
    return hipErrorInvalidValue;
}

hipError_t launch_pass_b_v3(const DevView& v, hipStream_t s) {
#define OCEAN_B3(NN)                                                              \
    case NN:                                                                      \
        return v.planes == 4 ? go_b3<NN, 4>(v, s) : go_b3<NN, 2>(v, s);
    switch (v.n) {
        OCEAN_B3(16)
        OCEAN_B3(32)
        OCEAN_B3(64)
        OCEAN_B3(128)
        OCEAN_B3(256)
        OCEAN_B3(512)
        OCEAN_B3(1024)
    }
#undef OCEAN_B3
    return hipErrorInvalidValue;
}

}  // namespace ocean
