// v3 fused frame for N <= 1024 (BASELINE cfg2 / cfg3 / cfg4 sizes).
//
// Pass A (k_pass_a3): evolve + row IFFT.  A workgroup owns RB = 1024/N
//   consecutive rows and all P planes of them (256 lanes for P = 4).  The
//   Stockham plan starts with radix R0 = 16/P so that in stage 0 one lane holds
//   every plane of R0 texels: the lane evolves those texels
//   (TimeDependentSpectrum.compute:20-47) and runs the first butterflies on
//   the results in registers -- no LDS round trip for the evolve.  The wave
//   data (kx, 1/|k|, kz, omega) is recomputed from (x, y, cascade) with the
//   init kernel's own arithmetic (spectrum_math.h wave_data, bit-identical)
//   instead of being read: 16 B/texel less HBM traffic.  Outputs go to the
//   column-tile-major intermediate [p][u][x/W][y][W], W = col_tile(N)
//   (64 B runs at N = 1024; 2-row workgroups that write 128 B runs measured
//   slower: this pass is VALU/latency-bound, not store-bound).
// Pass B (k_pass_b3): per W-column tile, column IFFT of each plane from one
//   contiguous 8*W*N-byte block, permute, fill/foam epilogue; the foam state
//   is a compact float in the same tile-major layout (4 B read + 4 B write
//   instead of a 16 B RGBA read), TURB is written as its broadcast image.
//
// Bytes per texel-cascade (P = 4): pass A 16 (h0) + 32 (planes) = 48;
// pass B 32 (planes) + 4 + 4 (foam) + 48 (DISP, DERIV, TURB) = 88.
#include <cstdlib>

#include "fft_engine.h"
#include "spectrum_math.h"

namespace ocean {
namespace {

constexpr int pa3_rows(int N, int RS = 2) { return N >= 1024 * RS ? 1 : 1024 * RS / N; }

// RS: row-sets per workgroup (RB = pa3_rows(N, RS) rows); PF: prefetch the
// next item's h0 before this item's transform (its loads are then ahead of
// this item's stores in the in-order vmcnt queue, so waiting for them never
// waits for the stores); NOSTORE: timing experiment only (no output).
template <int N, int P, int RS, bool PF, bool NOSTORE = false, bool NT = false>
__global__ __launch_bounds__(pa3_rows(N, RS) * P * N / kElems) void k_pass_a3(DevView v, float time, int total_rows) {
    constexpr int RB = pa3_rows(N, RS);
    constexpr int FIRST = 16 / P;
    using TW = StageTw<N, FIRST>;
    using E = Engine<N, RB * P, false, true, FIRST>;
    constexpr int T = E::THREADS;
    constexpr int R0 = E::R0;             // = FIRST (texels per lane)
    constexpr int NJ = N / R0;            // stage-0 butterflies per sequence
    constexpr int W = col_tile(N);
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
    int item = blockIdx.x;
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
        const WaveBand wb = band[u % v.C];
        float2 in[kElems];
#pragma unroll
        for (int r = 0; r < R0; ++r) {
            const Planes4 o = evolve_texel(h[r], wave_data(j + r * NJ, y, N, wb, v.gravity), time);
#pragma unroll
            for (int m = 0; m < P; ++m) in[m * R0 + r] = o.p[m];
        }
        // outputs: sequence b = p*RB + rr', element x -> tplane[p][u'][x/W][y'][x%W]
        auto emit = [&](int m, int q, float2 val) {
            if constexpr (NOSTORE) {
                asm volatile("" ::"v"(val.x), "v"(val.y));
                return;
            }
            int b, jj;
            E::template bj<E::RL>((int)threadIdx.x + m * T, b, jj);
            const int p = b / RB, r2 = b % RB;
            const int row2 = item * RB + r2;
            if (row2 < total_rows) {
                const int u2 = row2 / N, y2 = row2 % N;
                float2* rowp = v.tplane + (size_t)p * v.plane_stride + ((size_t)u2 * TILES * N + y2) * W;
                if constexpr (NSL % W == 0) {
                    // x = jj + q*NSL: x/W = jj/W + q*NSL/W, x%W = jj%W (compile-time tile stride)
                    float2* dst = rowp + (size_t)(jj / W) * N * W + (jj % W) + (size_t)q * (NSL / W) * N * W;
                    if constexpr (NT) store2_nt(dst, val);
                    else *dst = val;
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
        if constexpr (!PF) {
            if (next < items) load(next, h);
        }
    }
}

// Pass B: one item = (unit, W-column tile); planes in the order DyDxz, DxDz,
// DxxDzz, DyxDyz with the next PFD planes prefetched into registers.
template <int N, int P, int PFD = 1, int NT = 1>
__global__ __launch_bounds__(col_tile(N) * N / kElems) void k_pass_b3(DevView v, int items) {
    using CT = ColTile<N>;
    using E = typename CT::E;
    using TW = StageTw<N>;
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
    auto win16 = [&](const float4* base, int item) {
        const int u = item / CT::tiles, x0 = (item % CT::tiles) * W;
        return make_win(base + (size_t)u * N * N + x0, (unsigned)((N * N - x0) * 16));
    };
    auto load = [&](int item, int p, float2 (&d)[kElems]) {
        const Win w = make_win(v.tplane + (size_t)p * v.plane_stride + (size_t)item * TILE, TILE * 8);
#pragma unroll
        for (int i = 0; i < kElems; ++i) d[i] = bload2<(NT & 4) ? 2 : 0>(w, toff * 8, CT::in_dy(i) * W * 8);
    };

    // PFD planes in flight ahead of the one being transformed (register ring)
    float2 cur[kElems], nxt[kElems], nx2[PFD > 1 ? kElems : 1];
    int item = blockIdx.x;
    if (item < items) {
        load(item, order[0], cur);
        if constexpr (PFD > 1) load(item, order[1], nxt);
    }
    __syncthreads();
    for (; item < items; item += gridDim.x) {
        const int x0 = (item % CT::tiles) * W;
        float* foam = v.foam + (size_t)item * TILE + toff;
#pragma unroll
        for (int pi = 0; pi < P; ++pi) {
            const int p = order[pi];
            if constexpr (PFD > 1) {
                if (pi + 2 < P) load(item, order[pi + 2], nx2);
                else if (item + (int)gridDim.x < items) load(item + gridDim.x, order[pi + 2 - P], nx2);
            } else {
                if (pi + 1 < P) load(item, order[pi + 1], nxt);
                else if (item + (int)gridDim.x < items) load(item + gridDim.x, order[0], nxt);
            }
            float fb[kElems];
            if (p == 3) {
                const Win rf = make_win(v.foam + (size_t)item * TILE, TILE * 4);
#pragma unroll
                for (int m = 0; m < kElems / RL; ++m)
#pragma unroll
                    for (int q = 0; q < RL; ++q) fb[m * RL + q] = bload1(rf, toff * 4, CT::out_dy(m, q) * W * 4);
            }
            const Win wd = win16(v.disp, item), wt = win16(v.turb, item), wv = win16(v.deriv, item);
            // NT bit 0: texture outputs streamed (nontemporal); bit 1: foam state too;
            // bit 2: intermediate tile loads nontemporal
            auto st4 = [&](float4 x, const Win& w, int voff, int soff) {
                if constexpr (NT & 1) gstore4_nt(x, w, voff, soff);
                else gstore4(x, w, voff, soff);
            };
            auto stf = [&](float* a, float x) {
                if constexpr (NT & 2) store1_nt(a, x);
                else *a = x;
            };
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
                    if (v.normals) st4(normal_from_deriv(re, im, k.x, k.y), win16(v.normal, item), voff16, so);
                }
            };
            E::run_regs(cur, lds, tws, emit);
#pragma unroll
            for (int i = 0; i < kElems; ++i) {
                cur[i] = nxt[i];
                if constexpr (PFD > 1) nxt[i] = nx2[i];
            }
            __syncthreads();
        }
    }
}

int env_int(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return e ? std::atoi(e) : dflt;
}

int num_cus3() {
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
int grid3(K kernel, int threads, int items) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu <= 0)
        per_cu = 1;
    const int g = num_cus3() * per_cu;
    return items < g ? items : g;
}

template <int N, int P, int RS, bool PF, bool NOSTORE = false, bool NT = false>
hipError_t go_a3k(const DevView& v, float t, hipStream_t s) {
    constexpr int RB = pa3_rows(N, RS);
    constexpr int T = RB * P * N / kElems;
    const int total = v.units * N;
    const int items = (total + RB - 1) / RB;
    const int g = grid3(k_pass_a3<N, P, RS, PF, NOSTORE, NT>, T, items);
    hipLaunchKernelGGL((k_pass_a3<N, P, RS, PF, NOSTORE, NT>), dim3(g), dim3(T), 0, s, v, t, total);
    return hipGetLastError();
}

// OCEAN_A3_VARIANT selects measured alternatives at N = 1024 (pass A).
template <int N, int P>
hipError_t go_a3(const DevView& v, float t, hipStream_t s) {
    static const int variant = env_int("OCEAN_A3_VARIANT", 0);
    if constexpr (N == 1024 && P == 4) {
        switch (variant) {
            case 1: return go_a3k<N, P, 1, false>(v, t, s);       // 1 row / WG, no prefetch
            case 2: return go_a3k<N, P, 1, true>(v, t, s);        // 1 row / WG, prefetch
            case 11: return go_a3k<N, P, 2, true, true>(v, t, s);  // timing only: no stores
            case 3: return go_a3k<N, P, 2, true, false, true>(v, t, s);  // nontemporal intermediate stores
            default: return go_a3k<N, P, 2, true>(v, t, s);       // 2 rows / WG (512 lanes), prefetch
        }
    }
    return go_a3k<N, P, 1, false>(v, t, s);
}

template <int N, int P, int PFD, int NT = 1>
hipError_t go_b3k(const DevView& v, hipStream_t s) {
    constexpr int W = col_tile(N);
    constexpr int T = W * N / kElems;
    const int items = v.units * (N / W);
    const int g = grid3(k_pass_b3<N, P, PFD, NT>, T, items);
    hipLaunchKernelGGL((k_pass_b3<N, P, PFD, NT>), dim3(g), dim3(T), 0, s, v, items);
    return hipGetLastError();
}

// Two planes in flight at N = 1024 (one workgroup per CU, registers to spare):
// -3..5 % pass-B time on MI355X; OCEAN_B3_PFD=1 restores one.
template <int N, int P>
hipError_t go_b3(const DevView& v, hipStream_t s) {
    static const int pfd = env_int("OCEAN_B3_PFD", 2);
    static const int nt = env_int("OCEAN_B3_NT", 1);
    if constexpr (N == 1024) {
        if (pfd > 1) {
            if (nt == 0) return go_b3k<N, P, 2, 0>(v, s);
            if (nt == 3) return go_b3k<N, P, 2, 3>(v, s);
            if (nt == 5) return go_b3k<N, P, 2, 5>(v, s);
            if (nt == 7) return go_b3k<N, P, 2, 7>(v, s);
            return go_b3k<N, P, 2, 1>(v, s);
        }
    }
    return go_b3k<N, P, 1>(v, s);
}

}  // namespace

bool pass_v3_supported(int n) { return n >= 16 && n <= 1024; }

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
