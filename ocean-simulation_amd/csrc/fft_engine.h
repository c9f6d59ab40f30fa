// FFT engine shared by fft2.hip, fft3.hip and fft4k.hip: memory-op helpers, per-stage
// twiddle tables, the LDS Stockham engine and the column-tile geometry.
// DESIGN.md section 3 has the design notes.
#pragma once

#include <type_traits>

#include "fft_core.h"
#include "ocean_internal.h"

namespace ocean {
namespace {
using namespace fftcore;

// ---------------------------------------------------------- memory ops
// Stores go through plain global stores: on gfx950 / ROCm 7.2 the raw
// buffer_store_dwordx4 path with a scalar soffset produced corrupted texels
// (store data VGPRs overwritten by the following VALU before the store read
// them; reproduced with tools/dbg_passb.py, loads unaffected) -- DESIGN.md.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
typedef unsigned int u32x4 __attribute__((__vector_size__(4 * sizeof(unsigned int))));

// A texture window: buffer descriptor (loads) + base pointer (stores).
struct Win {
    rsrc_t r;
    char* p;
};
__device__ __forceinline__ Win make_win(const void* base, unsigned bytes) {
    Win w;
    w.r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
    w.p = (char*)const_cast<void*>(base);
    return w;
}
template <int AUX = 0>  // AUX = 2: nontemporal (streamed, read-once data)
__device__ __forceinline__ float2 bload2(const Win& w, int voff, int soff) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(w.r, voff, soff, AUX);
    return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
}
__device__ __forceinline__ float4 bload4(const Win& w, int voff, int soff) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(w.r, voff, soff, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
__device__ __forceinline__ float bload1(const Win& w, int voff, int soff) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(w.r, voff, soff, 0));
}
// Byte offsets are non-negative and < 4 GiB: as an unsigned 32-bit lane offset from the window's
// scalar base the store can take the saddr form (SGPR base + VGPR offset) instead of a 64-bit VALU
// address add per store (pass BQ: 68 -> 30 such adds; frame time unchanged, A/B round 3).
typedef unsigned store_off_t;
__device__ __forceinline__ void gstore2(float2 x, const Win& w, int voff, int soff) {
    *(float2*)(w.p + (store_off_t)(voff + soff)) = x;
}
__device__ __forceinline__ void gstore4(float4 x, const Win& w, int voff, int soff) {
    *(float4*)(w.p + (store_off_t)(voff + soff)) = x;
}
// Streaming (nontemporal) stores for outputs nothing in the frame reads back:
// measured on the pass-B access shape (tools/membench.hip) 7.1 TB/s against
// 5.8 TB/s with default-policy stores -- the write stream stops evicting the
// tile reads' lines.
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void gstore4_nt(float4 x, const Win& w, int voff, int soff) {
    const f32x4 v = {x.x, x.y, x.z, x.w};
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(w.p + (store_off_t)(voff + soff)));
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void gstore2_nt(float2 x, const Win& w, int voff, int soff) {
    const f32x2 v = {x.x, x.y};
    __builtin_nontemporal_store(v, reinterpret_cast<f32x2*>(w.p + (store_off_t)(voff + soff)));
}
__device__ __forceinline__ void store4_nt(float4* p, float4 x) {
    const f32x4 v = {x.x, x.y, x.z, x.w};
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
}

// ------------------------------------------------------------- twiddles
// Per-stage tables, stage s >= 1 (Ns, R): entry r*Ns + k = exp(+2 pi i r k / (Ns R)),
// k < Ns, r < R (r-major: lanes with consecutive k read consecutive entries,
// bank-conflict free; a butterfly's R-1 twiddles sit at compile-time strides);
// stages concatenated.  Built on the host in double precision
// at tw + N + 128 (ocean_abi.cpp).
template <int N, int R0 = 16>
struct StageTw {
    static constexpr int S = n_stages(N, R0);
    static constexpr int off(int s) {
        return s <= 1 ? 0 : off(s - 1) + ns_of(N, s - 1, R0) * radix_of(N, s - 1, R0);
    }
    static constexpr int kEntries = off(S) > 0 ? off(S) : 1;
    static constexpr bool kInLds = kEntries * 8 <= 20 * 1024;
    static constexpr int kLdsEntries = kInLds ? kEntries : 1;
    // table sets for R0 = 16, 8, 4 follow each other at tw + N + 128
    static constexpr int base() {
        return R0 == 16 ? 0
                        : (R0 == 8 ? StageTw<N, 16>::off(n_stages(N, 16))
                                   : StageTw<N, 16>::off(n_stages(N, 16)) + StageTw<N, 8>::off(n_stages(N, 8)));
    }
    static __device__ __forceinline__ const float2* global_table(const float2* tw) {
        constexpr int B = base();  // forced constant: a runtime call of the recursive constexpr otherwise
        return tw + N + 128 + B;
    }
    static __device__ __forceinline__ void load(float2* lds, const float2* __restrict__ tw, int tid, int nthreads) {
        if constexpr (kInLds) {
            const float2* src = global_table(tw);
            for (int i = tid; i < kEntries; i += nthreads) lds[i] = src[i];
        }
    }
    // table to read from: the LDS copy when it fits, else global memory (L1/L2 resident)
    static __device__ __forceinline__ const float2* table(const float2* lds, const float2* tw) {
        if constexpr (kInLds) return lds;
        else return global_table(tw);
    }
    // twiddle the R inputs of butterfly j of stage ST (v[0] never needs one)
    template <int ST>
    static __device__ __forceinline__ void apply(float2* v, int j, const float2* tws) {
        constexpr int R = radix_of(N, ST, R0), NS = ns_of(N, ST, R0);
        if constexpr (NS > 1) {
            constexpr int O = off(ST);
            const float2* t = tws + O + (j & (NS - 1));
#pragma unroll
            for (int r = 1; r < R; ++r) v[r] = cmul(v[r], t[r * NS]);
        }
    }
};

// Compact variant for N >= 2048, where the full tables do not fit beside a
// whole-row LDS image: a stage with Ns >= 16 keeps only the rows r = 1, 2, 4,
// 8 of its table (exact, from the double-precision global table) and forms
// w^r for the other r as products of those (w^3 = w^2 w, w^13 = w^8 w^5, ...:
// at most three roundings deep, a few ulp).  N = 4096, first radix 4: 18.5 KiB
// instead of 41 KiB.  Reading the full table from global memory instead puts
// twiddle loads behind the previous item's stores in the in-order vmcnt queue.
template <int N, int R0>
struct StageTwCompact {
    using Full = StageTw<N, R0>;
    static constexpr int S = n_stages(N, R0);
    static constexpr bool compact(int s) { return ns_of(N, s, R0) >= 16 && radix_of(N, s, R0) >= 2; }
    static constexpr int rows(int s) { return compact(s) ? ilog2(radix_of(N, s, R0)) : radix_of(N, s, R0); }
    static constexpr int off(int s) { return s <= 1 ? 0 : off(s - 1) + ns_of(N, s - 1, R0) * rows(s - 1); }
    static constexpr int kEntries = off(S) > 0 ? off(S) : 1;
    static constexpr bool kInLds = true;
    static constexpr int kLdsEntries = kEntries;
    static_assert(kEntries * 8 <= 32 * 1024, "compact twiddles must fit LDS");
    template <int s>
    static __device__ __forceinline__ void load_stage(float2* lds, const float2* src, int tid, int nthreads) {
        if constexpr (s < S) {
            constexpr int NS = ns_of(N, s, R0), RW = rows(s), O = off(s), FO = Full::off(s);
            constexpr bool CP = compact(s);
            for (int i = tid; i < NS * RW; i += nthreads) {
                const int row = i / NS, k = i % NS;
                const int r = CP ? (1 << row) : row;
                lds[O + i] = src[FO + r * NS + k];
            }
            load_stage<s + 1>(lds, src, tid, nthreads);
        }
    }
    static __device__ __forceinline__ void load(float2* lds, const float2* __restrict__ tw, int tid, int nthreads) {
        load_stage<1>(lds, Full::global_table(tw), tid, nthreads);
    }
    static __device__ __forceinline__ const float2* table(const float2* lds, const float2*) { return lds; }
    template <int ST>
    static __device__ __forceinline__ void apply(float2* v, int j, const float2* tws) {
        constexpr int R = radix_of(N, ST, R0), NS = ns_of(N, ST, R0);
        if constexpr (NS > 1) {
            constexpr int O = off(ST);
            const float2* t = tws + O + (j & (NS - 1));
            if constexpr (compact(ST)) {
                float2 w[R];
#pragma unroll
                for (int b = 0; (1 << b) < R; ++b) w[1 << b] = t[b * NS];
#pragma unroll
                for (int r = 3; r < R; ++r) {
                    if ((r & (r - 1)) != 0) {
                        int hb = 1;
                        while (hb * 2 <= r) hb *= 2;
                        w[r] = cmul(w[hb], w[r - hb]);
                    }
                }
#pragma unroll
                for (int r = 1; r < R; ++r) v[r] = cmul(v[r], w[r]);
            } else {
#pragma unroll
                for (int r = 1; r < R; ++r) v[r] = cmul(v[r], t[r * NS]);
            }
        }
    }
};

// The compact tables of an L-point plan (R0 first) inside a context of size N > L, built from the
// context's base table tw[m] = exp(2 pi i m / N) (the per-stage global tables are the N-point
// plan's): entry (s, r, k) = tw[r k N / (Ns R)].  Pass A3P (fftq.hip) runs 2048-point transforms
// in a 4096 context.
template <int L, int N, int R0>
struct StageTwCompactSub : StageTwCompact<L, R0> {
    using Base = StageTwCompact<L, R0>;
    template <int s>
    static __device__ __forceinline__ void load_stage(float2* lds, const float2* tw, int tid, int nthreads) {
        if constexpr (s < Base::S) {
            constexpr int NS = ns_of(L, s, R0), R = radix_of(L, s, R0), RW = Base::rows(s), O = Base::off(s);
            constexpr bool CP = Base::compact(s);
            for (int i = tid; i < NS * RW; i += nthreads) {
                const int row = i / NS, k = i % NS;
                const int r = CP ? (1 << row) : row;
                lds[O + i] = tw[(r * k * (N / (NS * R))) & (N - 1)];
            }
            load_stage<s + 1>(lds, tw, tid, nthreads);
        }
    }
    static __device__ __forceinline__ void load(float2* lds, const float2* __restrict__ tw, int tid, int nthreads) {
        load_stage<1>(lds, tw, tid, nthreads);
    }
};

// Per-stage tables of an L-point plan inside a context of size N >= L, read from the context's base table
// tw[m] = exp(2 pi i m / N): entry r*Ns + k = tw[r k N / (Ns R)] (the same float bits as StageTw<L>'s
// double-rounded entries).  The 4096 operator's 2048-point columns and the four-step passes use it.
template <int L, int N>
struct SubTw {
    using Full = StageTw<L, 16>;
    static constexpr int S = Full::S;
    static constexpr int kEntries = Full::kEntries;
    static constexpr int kLdsEntries = kEntries;
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

// LDS twiddle tables for plan (N, R0): the full per-stage tables when they fit, else the compact form.
template <int N, int R0 = 16>
using StageTwLds = std::conditional_t<StageTw<N, R0>::kInLds, StageTw<N, R0>, StageTwCompact<N, R0>>;

// --------------------------------------------------------------- engine
// A workgroup transforms B sequences of length N with THREADS = B*N/EL
// lanes, EL (16, or 32: two butterflies) complex values per lane per stage.  Lane -> (sequence b,
// butterfly j) is b-fastest (SEQ_FAST, column tiles) or j-fastest (rows).
// Stage-0 input slot m*R0 + r is element y = j_m + r*N/R0 of sequence b_m;
// last-stage output slot (m, q) is element y = j_m + q*N/RL.
// SUB: the workgroup runs several engines side by side, THREADS lanes each (a power of two); a lane
// works in engine threadIdx.x / THREADS as lane threadIdx.x % THREADS.
template <int N, int B, bool SEQ_FAST, bool PAD, int FIRST = 16, class TWT = StageTw<N, FIRST>, int EL = kElems,
          bool SUB = false>
struct Engine {
    static constexpr int ELEMS = EL;  // complex values per lane per stage (16, or 32 for two butterflies of 16)
    static constexpr int THREADS = B * N / EL;
    static_assert(!SUB || (THREADS & (THREADS - 1)) == 0, "side-by-side engines need a power-of-two lane count");
    static __device__ __forceinline__ int lane() { return SUB ? (int)(threadIdx.x & (THREADS - 1)) : (int)threadIdx.x; }
    static constexpr int S = n_stages(N, FIRST);
    static constexpr int R0 = radix_of(N, 0, FIRST);
    static constexpr int RL = radix_of(N, S - 1, FIRST);
    static constexpr int LDS_ELEMS = PAD ? padded(B * N) : B * N;

    template <int R>
    static __device__ __forceinline__ void bj(int g, int& b, int& j) {
        if constexpr (SEQ_FAST) {
            b = g % B;
            j = g / B;
        } else {
            b = g / (N / R);
            j = g % (N / R);
        }
    }
    static __device__ __forceinline__ int raw(int b, int y) { return SEQ_FAST ? y * B + b : b * N + y; }
    // Padding.  Rows (b-major): one slot every 16 elements, i + i/16.  Column
    // tiles (SEQ_FAST, y-major [y][B]): one B-row every 16 rows,
    // i + (i / 16B) * B -- the radix-16 stage-0 write (rows 16j + q, q < 16)
    // then spreads the lanes' j over the banks instead of a 16*B*8-byte
    // stride that maps them all to one bank group.
    static __device__ __forceinline__ int lidx(int b, int y) {
        const int i = raw(b, y);
        return !PAD ? i : (SEQ_FAST ? i + (i / (16 * B)) * B : pad(i));
    }
    // LDS offset of the k-th element at raw-index stride rs from a butterfly's
    // base element, at compile time: pad(base + k*rs) = pad(base) + loff(k, rs).
    // Rows: every access pattern has power-of-two strides with the base placed
    // so that (base % 16) + (k*rs % 16) < 16.  Column tiles: the row stride is
    // a multiple of 16, or 1 from a 16-aligned base (seq_pad_ok()).
    static constexpr int loff(int k, int rs) {
        return !PAD ? k * rs : (SEQ_FAST ? k * rs + ((k * rs) / (16 * B)) * B : k * rs + (k * rs) / 16);
    }
    static constexpr bool seq_pad_ok() {
        for (int s = 0; s < S; ++s) {
            const int R = radix_of(N, s, FIRST), NS = ns_of(N, s, FIRST);
            if (!((N / R) % 16 == 0 || N / R == 1)) return false;  // reads: rows j + r N/R
            if (!(NS == 1 || NS % 16 == 0)) return false;           // writes: rows y0 + q NS
            if (NS == 1 && R > 16) return false;
        }
        return true;
    }
    static_assert(!(PAD && SEQ_FAST) || seq_pad_ok(), "column-tile padding needs 16-row-aligned strides");
    static constexpr bool linear() { return true; }
    // Stages st.. are wave-private when every one of them has N / R = 64 butterflies
    // per sequence on row-major lanes: lane g = tid + m * THREADS then works on sequence
    // g / 64, so each wave reads and writes only its own sequences (the same ones at
    // every such stage) and the stages need no workgroup barrier -- LDS operations of
    // one wave execute in order; a compiler fence keeps them in program order.
    static constexpr bool wave_private(int st) {
        if (SEQ_FAST) return false;
        for (int s = st; s < S; ++s)
            if (N / radix_of(N, s, FIRST) != 64) return false;
        return st < S;
    }
    template <int ST>
    static __device__ __forceinline__ void stage_sync() {
        if constexpr (wave_private(ST)) __asm__ volatile("" ::: "memory");
        else __syncthreads();
    }

    // Stages ST.. from LDS; the last stage hands (m, q, value) to emit.  Butterflies of sequences
    // b >= live or b < lo are skipped (their lanes still join the stage barriers): an image with idle
    // sequence slots.
    template <int ST, class Emit>
    static __device__ __forceinline__ void stages_from(float2* lds, const float2* tws, Emit& emit, int live = B,
                                                       int lo = 0) {
        constexpr int R = radix_of(N, ST, FIRST);
        constexpr int NS = ns_of(N, ST, FIRST);
        constexpr int BF = EL / R;
        constexpr bool LAST = (ST == S - 1);
        constexpr int RD = (SEQ_FAST ? B : 1) * (N / R);  // raw stride between a butterfly's inputs
        constexpr int WR = (SEQ_FAST ? B : 1) * NS;       // raw stride between its outputs
        float2 v[EL];
#pragma unroll
        for (int m = 0; m < BF; ++m) {
            int b, j;
            bj<R>(lane() + m * THREADS, b, j);
            if (b >= live || b < lo) continue;
            if constexpr (linear()) {
                const float2* src = lds + lidx(b, j);
#pragma unroll
                for (int r = 0; r < R; ++r) v[m * R + r] = src[loff(r, RD)];
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) v[m * R + r] = lds[lidx(b, j + r * (N / R))];
            }
        }
        if constexpr (!LAST) stage_sync<ST>();
#pragma unroll
        for (int m = 0; m < BF; ++m) {
            int b, j;
            bj<R>(lane() + m * THREADS, b, j);
            if (b >= live || b < lo) continue;
            TWT::template apply<ST>(&v[m * R], j, tws);
            Idft<R>::run(&v[m * R]);
            if constexpr (LAST) {
#pragma unroll
                for (int q = 0; q < R; ++q) emit(m, q, v[m * R + q]);
            } else {
                const int y0 = (j / NS) * NS * R + (j & (NS - 1));
                if constexpr (linear()) {
                    float2* dst = lds + lidx(b, y0);
#pragma unroll
                    for (int q = 0; q < R; ++q) dst[loff(q, WR)] = v[m * R + q];
                } else {
#pragma unroll
                    for (int q = 0; q < R; ++q) lds[lidx(b, y0 + q * NS)] = v[m * R + q];
                }
            }
        }
        if constexpr (!LAST) {
            stage_sync<ST>();
            stages_from<ST + 1>(lds, tws, emit, live, lo);
        }
    }

    // Stage-0 outputs of butterfly m to LDS (Ns = 1: y = R0 j + q).
    static __device__ __forceinline__ void stage0_store(float2* lds, int m, const float2* v) {
        int b, j;
        bj<R0>(lane() + m * THREADS, b, j);
        if constexpr (linear()) {
            float2* dst = lds + lidx(b, j * R0);
#pragma unroll
            for (int q = 0; q < R0; ++q) dst[loff(q, SEQ_FAST ? B : 1)] = v[q];
        } else {
#pragma unroll
            for (int q = 0; q < R0; ++q) lds[lidx(b, j * R0 + q)] = v[q];
        }
    }

    // Full transform from registers (stage-0 layout); LDS free on entry.
    template <class Emit>
    static __device__ __forceinline__ void run_regs(float2 (&v)[EL], float2* lds, const float2* tws, Emit& emit) {
        constexpr int BF = EL / R0;
#pragma unroll
        for (int m = 0; m < BF; ++m) Idft<R0>::run(&v[m * R0]);
        if constexpr (S == 1) {
#pragma unroll
            for (int m = 0; m < BF; ++m)
#pragma unroll
                for (int q = 0; q < R0; ++q) emit(m, q, v[m * R0 + q]);
        } else {
#pragma unroll
            for (int m = 0; m < BF; ++m) stage0_store(lds, m, &v[m * R0]);
            __syncthreads();
            stages_from<1>(lds, tws, emit);
        }
    }

    template <class Emit>
    static __device__ __forceinline__ void run_lds(float2* lds, const float2* tws, Emit& emit) {
        stages_from<0>(lds, tws, emit);
    }
};

__device__ __forceinline__ float perm_sign(int x, int y) { return ((x + y) & 1) ? -1.0f : 1.0f; }

// ------------------------------------------------------ column-tile I/O
// Column tile = W columns x N rows of one unit.  Lane (b, j) with b = tid % W,
// j = tid / W for every stage; element (b, y) of the tile lives at texel
// (x0 + b, y).  Stage-0 inputs are rows j + in_dy(r); last-stage outputs are
// rows j + out_dy(m, q): the lane's base texel plus compile-time offsets.
template <int N, int WW = col_tile(N)>
struct ColTile {
    static constexpr int W = WW;
    static constexpr int tiles = N / W;
    using TW = StageTwLds<N>;
    using E = Engine<N, W, true, Engine<N, W, true, false>::seq_pad_ok(), 16, TW>;
    static constexpr int T = E::THREADS;
    static constexpr int R0 = E::R0, RL = E::RL;
    static __device__ __forceinline__ int lane_b() { return (int)threadIdx.x % W; }
    static __device__ __forceinline__ int lane_j() { return (int)threadIdx.x / W; }
    static constexpr int out_dy(int m, int q) { return m * (T / W) + q * (N / RL); }
    static constexpr int in_dy(int r) { return r * (N / R0); }
};

}  // namespace
}  // namespace ocean
