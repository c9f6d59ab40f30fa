// Column passes for N = 2048 / 4096 (cfg5), four-step.
//
// At N = 4096 a column tile narrow enough for its whole columns to sit in LDS
// (4 columns, 128 KiB per plane) writes the output textures in 64-byte row
// pieces 64 KiB apart, and its intermediate rows are 32-byte pieces: measured
// (tools/membench4k.hip) 1.8 and 1.4 TB/s.  With N = L1 * L0, L1 = 64,
// y = y1 + L1 y0 and k = k0 + L0 k1 the column transform splits into
//   step 1: A[y1][k0] = w_N^(y1 k0) * sum_y0 X[y1 + L1 y0] w_L0^(y0 k0)
//   step 2: Y[k0 + L0 k1] = sum_y1 A[y1][k0] w_L1^(y1 k1)
// (w = exp(+2 pi i / .), the inverse transform of IFFT.compute).  Pass C1
// runs step 1 in place on the 16-column tile-major intermediate (A[y1][k0] in
// the slot of X[y1 + L1 k0]); pass C2 runs step 2 -- reading 64 consecutive
// rows per k0 -- and the permute + fill/foam epilogue of pass B, with 256-byte
// output row pieces.  Every access is a >= 128-byte contiguous piece; the cost
// is one extra read + write of the intermediate (64 B per texel-cascade).
#include "fft_engine.h"
#include "spectrum_math.h"

namespace ocean {
namespace {

constexpr int kL1 = 64;   // step-2 length
constexpr int kWT = 16;   // intermediate tile width (128-byte float2 rows)
constexpr int kSeq = 64;  // sequences per workgroup: 16 columns x 4 y1 (C1) or 4 k0 (C2)

// Pass C1: item = (plane, unit, 16-column tile, block of 4 y1).  Sequence
// b = y1_local * 16 + column, element y0: intermediate slot
// tile + (y1_0 * 16 + b) + y0 * (L1 * 16).  In place.
// Q (three-plane frame, fftq.hip): planes Q1..Q3; an item of Q1 also forms R[Q4] = i kz R[Q1] + d0
// (row 0: srow) from the loaded values and runs step 1 on it into the fourth plane slot.
template <int N, bool Q = false>
__global__ __launch_bounds__(kSeq * (N / kL1) / kElems) void k_col4s1(DevView v, int items) {
    constexpr int L0 = N / kL1;
    using CT = ColTile<L0, kSeq>;
    using E = Engine<L0, kSeq, true, Engine<L0, kSeq, true, false>::seq_pad_ok(), 16, SubTw<L0, N>>;
    using TW = SubTw<L0, N>;
    constexpr int T = E::THREADS;
    constexpr int TILE = N * kWT;             // elements per tile
    constexpr int BLKS = kL1 / (kSeq / kWT);  // y1 blocks per tile
    constexpr int ES = kL1 * kWT;             // element (y0) stride
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    __shared__ float2 two[128];  // two-level table of w_N^m: lo = m % 64, hi = m / 64
    __shared__ float dks[kMaxCascades];
    TW::load(twl, v.tw, threadIdx.x, T);
    for (int i = threadIdx.x; i < 128; i += T) two[i] = v.tw[N + i];
    if (Q && (int)threadIdx.x < v.C) dks[threadIdx.x] = 2.0f * kPi / v.casc[threadIdx.x * 5];  // wave_band's dk
    const int lb = (int)threadIdx.x % kSeq, lj = (int)threadIdx.x / kSeq;
    const int tiles = N / kWT;
    const int bt0 = v.x0 / kWT, bnt = v.nx / kWT;  // column band's tiles
    auto plane_of = [&](int item) { return item / BLKS / (v.units * bnt); };
    auto ut_of = [&](int item) {  // unit * tiles + tile
        const int ub = item / BLKS % (v.units * bnt);
        return (ub / bnt) * tiles + bt0 + ub % bnt;
    };
    auto base_at = [&](int item, int p) {
        return v.tplane + (size_t)p * v.inter_stride + (size_t)ut_of(item) * TILE + (item % BLKS) * (kSeq / kWT) * kWT;
    };
    auto base_of = [&](int item) { return base_at(item, plane_of(item)); };
    float2 cur[kElems], nxt[kElems];
    auto load = [&](int item, float2 (&d)[kElems]) {
        const float2* src = base_of(item) + lb + (size_t)lj * ES;
#pragma unroll
        for (int i = 0; i < kElems; ++i) d[i] = src[(size_t)CT::in_dy(i) * ES];
    };
    int item = blockIdx.x;
    if (item < items) load(item, cur);
    __syncthreads();
    for (; item < items; item += gridDim.x) {
        const int next = item + gridDim.x;
        if (next < items) load(next, nxt);
        float2* dst = base_of(item) + lb + (size_t)lj * ES;
        const int y1 = (item % BLKS) * (kSeq / kWT) + lb / kWT;
        const bool q1 = Q && plane_of(item) == 0;
        float2 q4[Q ? kElems : 1];
        if constexpr (Q) {
            if (q1) {  // R[Q4] of the lane's rows y = y1 + L1 y0 (y0 = lj + in_dy(i)) before cur is consumed
                const int ut = ut_of(item), u = ut / tiles;
                const float dk = dks[(u + v.c0) % v.C];
                const float2* side = v.qside + (size_t)u * 2 * N;
#pragma unroll
                for (int i = 0; i < kElems; ++i) {
                    const int y = y1 + kL1 * (lj + CT::in_dy(i));
                    const float kz = (float)(y - N / 2) * dk;
                    const float2 d = side[y], c = cur[i];
                    q4[i] = make_float2(d.x - kz * c.y, d.y + kz * c.x);
                }
                if (y1 == 0 && lj == 0) q4[0] = side[N + (ut % tiles) * kWT + lb % kWT];  // row 0: srow
            }
        }
        auto emit = [&](int m, int q, float2 val) {
            const int dy = CT::out_dy(m, q);
            const int mm = y1 * (lj + dy);  // < L1 * L0 = N
            const float2 w = cmul(two[mm & 63], two[64 + (mm >> 6)]);
            dst[(size_t)dy * ES] = cmul(val, w);
        };
        E::run_regs(cur, lds, twl, emit);
        if constexpr (Q) {
            if (q1) {
                __syncthreads();
                float2* dst4 = base_at(item, 3) + lb + (size_t)lj * ES;
                auto emit4 = [&](int m, int q, float2 val) {
                    const int dy = CT::out_dy(m, q);
                    const int mm = y1 * (lj + dy);
                    const float2 w = cmul(two[mm & 63], two[64 + (mm >> 6)]);
                    dst4[(size_t)dy * ES] = cmul(val, w);
                };
                E::run_regs(q4, lds, twl, emit4);
            }
        }
#pragma unroll
        for (int i = 0; i < kElems; ++i) cur[i] = nxt[i];
        __syncthreads();
    }
}

// Pass C2: item = (unit, 16-column tile, block of 4 k0).  Sequence b = k0_local
// * 16 + column, element y1 at slot tile + (L1 (k0_0 + k0_local)) * 16 + col +
// y1 * 16.  Output row k0 + L0 k1, column x0 + col; the four planes in the
// order DyDxz, DxDz, DxxDzz, DyxDyz as in pass B.
// Q (three-plane frame): slots 1, 0, 3, 2 hold R[Q2], R[Q1], R[Q4], R[Q3] after step 1, whose
// transforms are (Dy, Dyx), (Dx, Dz), (Dxz, Dzz), (Dyz, Dxx) (fftq.hip, pass BQ's epilogue).
template <int N, int P, bool Q = false>
__global__ __launch_bounds__(kSeq * kL1 / kElems) void k_col4s2(DevView v, int items) {
    constexpr int L0 = N / kL1;
    using CT = ColTile<kL1, kSeq>;
    using E = Engine<kL1, kSeq, true, Engine<kL1, kSeq, true, false>::seq_pad_ok(), 16, SubTw<kL1, N>>;
    using TW = SubTw<kL1, N>;
    constexpr int T = E::THREADS;
    constexpr int RL = E::RL;
    constexpr int TILE = N * kWT;
    constexpr int K0B = kSeq / kWT;           // k0 per item
    constexpr int BLKS = L0 / K0B;            // k0 blocks per tile
    __shared__ float2 lds[E::LDS_ELEMS];
    __shared__ float2 twl[TW::kLdsEntries];
    __shared__ float2 keep[kElems * T];
    TW::load(twl, v.tw, threadIdx.x, T);
    constexpr int order[4] = {1, 0, 3, 2};
    const int lb = (int)threadIdx.x % kSeq, lj = (int)threadIdx.x / kSeq;
    const int col = lb % kWT, k0l = lb / kWT;
    const int tiles = N / kWT;
    auto kput = [&](int i, float2 x) { keep[i * T + threadIdx.x] = x; };
    auto kget = [&](int i) { return keep[i * T + threadIdx.x]; };
    const int bt0 = v.x0 / kWT, bnt = v.nx / kWT;  // column band's tiles
    auto full = [&](int ub) { return (ub / bnt) * tiles + bt0 + ub % bnt; };
    auto load = [&](int item, int p, float2 (&d)[kElems]) {
        const int blk = item % BLKS, ut = full(item / BLKS);
        const float2* src = v.tplane + (size_t)p * v.inter_stride + (size_t)ut * TILE +
                            (size_t)kL1 * (blk * K0B + k0l) * kWT + col + lj * kWT;
#pragma unroll
        for (int i = 0; i < kElems; ++i) d[i] = src[CT::in_dy(i) * kWT];
    };
    float2 cur[kElems], nxt[kElems];
    int item = blockIdx.x;
    if (item < items) load(item, order[0], cur);
    __syncthreads();
    for (; item < items; item += gridDim.x) {
        const int blk = item % BLKS, ut = full(item / BLKS);
        const int u = ut / tiles, tile = ut % tiles;
        const int k0 = blk * K0B + k0l, x = tile * kWT + col;
        const int y0 = k0 + L0 * lj;  // lane's first output row; element (m, q) adds L0 * out_dy
        float* foam = v.foam + (size_t)ut * TILE + col + (size_t)y0 * kWT;  // tile-major [u][x/16][y][16]
        const size_t t0 = ((size_t)u * N + y0) * N + x;
        float4 *disp = v.disp + t0, *turb = v.turb + t0, *deriv = v.deriv + t0, *nrm = v.normal + t0;
        float fb[kElems];
        float kreg[Q ? kElems : 1];
#pragma unroll
        for (int pi = 0; pi < P; ++pi) {
            const int p = order[pi];
            if (pi + 1 < P && order[pi + 1] == (Q ? 2 : 3)) {  // foam state, one step ahead
#pragma unroll
                for (int m = 0; m < kElems / RL; ++m)
#pragma unroll
                    for (int q = 0; q < RL; ++q)
                        fb[m * RL + q] = foam[(size_t)L0 * CT::out_dy(m, q) * kWT];
            }
            if (pi + 1 < P) load(item, order[pi + 1], nxt);
            else if (item + (int)gridDim.x < items) load(item + gridDim.x, order[0], nxt);
            auto emit = [&](int m, int q, float2 val) {
                const int i = m * RL + q;
                const int dy = CT::out_dy(m, q);
                const float s = perm_sign(x * v.xstr + v.xpar, y0 + L0 * dy);  // x: compact column under a parity
                const float re = val.x * s, im = val.y * s;
                const size_t to = (size_t)L0 * dy * N;  // compile-time row offset
                if constexpr (Q) {
                    if (p == 1) {  // (Dy, Dyx)
                        kput(i, make_float2(re, im));
                    } else if (p == 0) {  // (Dx, Dz): DISP
                        const float2 k = kget(i);
                        store4_nt(disp + to, make_float4(re, k.x, im, 1.0f));
                        kreg[i] = k.y;
                    } else if (p == 3) {  // (Dxz, Dzz)
                        kput(i, make_float2(re, im));
                    } else {  // (Dyz, Dxx): foam, TURB, DERIV, NORMAL
                        const float2 k = kget(i);
                        const float f = foam_update(fb[i], im, k.y, k.x);
                        // the foam state (256 MiB at cfg5) is read back only next frame: nontemporal
                        // (cfg5 447-448 -> 450-451 frames/s; cfg3 / cfg4 keep theirs cached, log section 8)
                        __builtin_nontemporal_store(f, &foam[(size_t)L0 * dy * kWT]);
                        store4_nt(turb + to, make_float4(f, f, f, f));
                        store4_nt(deriv + to, make_float4(kreg[i], re, im, k.y));
                        if (v.normals) store4_nt(nrm + to, normal_from_deriv(kreg[i], re, im, k.y));
                    }
                    return;
                }
                if (p == 1) {
                    kput(i, make_float2(re, im));
                } else if (p == 0) {
                    store4_nt(disp + to, make_float4(re, kget(i).x, im, 1.0f));
                } else if (p == 3) {
                    const float f = foam_update(fb[i], re, im, kget(i).y);
                    foam[(size_t)L0 * dy * kWT] = f;
                    store4_nt(turb + to, make_float4(f, f, f, f));
                    kput(i, make_float2(re, im));
                } else {
                    const float2 k = kget(i);
                    store4_nt(deriv + to, make_float4(re, im, k.x, k.y));
                    if (v.normals) store4_nt(nrm + to, normal_from_deriv(re, im, k.x, k.y));
                }
            };
            E::run_regs(cur, lds, twl, emit);
#pragma unroll
            for (int i = 0; i < kElems; ++i) cur[i] = nxt[i];
            __syncthreads();
        }
    }
}

template <class K>
int grid4(K kernel, int threads, int items, int max_per_cu = 0) {
    int per_cu = resident_per_cu((const void*)kernel, threads);
    if (max_per_cu > 0 && per_cu > max_per_cu) per_cu = max_per_cu;
    const int g = device_cus() * per_cu;
    return items < g ? items : g;
}

template <int N, bool Q = false>
hipError_t go_c1(const DevView& v, hipStream_t s) {
    constexpr int T = kSeq * (N / kL1) / kElems;
    const int items = (Q ? 3 : v.planes) * v.units * (v.nx / kWT) * (kL1 / (kSeq / kWT));
    // two workgroups per CU, not the four that fit: cfg5 column passes 1.72 -> 1.67 ms
    // (three per CU: 1.70 ms), docs/MEASUREMENTS.md section 3
    const int g = grid4(k_col4s1<N, Q>, T, items, 2);
    launch((k_col4s1<N, Q>), dim3(g), dim3(T), 0, s, v, items);
    return hipGetLastError();
}

template <int N, int P, bool Q = false>
hipError_t go_c2(const DevView& v, hipStream_t s) {
    constexpr int T = kSeq * kL1 / kElems;
    const int items = v.units * (v.nx / kWT) * ((N / kL1) / (kSeq / kWT));
    const int g = grid4(k_col4s2<N, P, Q>, T, items);
    launch((k_col4s2<N, P, Q>), dim3(g), dim3(T), 0, s, v, items);
    return hipGetLastError();
}

}  // namespace

bool pass_c4_supported(int n) { return n == 2048 || n == 4096; }

hipError_t launch_pass_c4q(const DevView& v, hipStream_t s) {
    if (v.planes != 4 || !v.qside) return hipErrorInvalidValue;
    if (v.n == 2048) {
        const hipError_t e = go_c1<2048, true>(v, s);
        return e != hipSuccess ? e : go_c2<2048, 4, true>(v, s);
    }
    if (v.n != 4096) return hipErrorInvalidValue;
    const hipError_t e = go_c1<4096, true>(v, s);
    return e != hipSuccess ? e : go_c2<4096, 4, true>(v, s);
}

hipError_t launch_pass_c4(const DevView& v, hipStream_t s) {
    hipError_t e = hipErrorInvalidValue;
    switch (v.n) {
        case 2048: e = go_c1<2048>(v, s); break;
        case 4096: e = go_c1<4096>(v, s); break;
    }
    if (e != hipSuccess) return e;
    switch (v.n) {
        case 2048: return v.planes == 4 ? go_c2<2048, 4>(v, s) : go_c2<2048, 2>(v, s);
        case 4096: return v.planes == 4 ? go_c2<4096, 4>(v, s) : go_c2<4096, 2>(v, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace ocean
