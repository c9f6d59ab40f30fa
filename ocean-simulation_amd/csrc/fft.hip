// Batched, centred, unnormalised 2D inverse FFT for gfx950 (complex64), plus
// the fused frame kernels.
//
// Reference operator: IFFT.InverseFastFourierTransform (IFFT.cs:66-94) =
// log2N radix-2 horizontal dispatches + log2N vertical dispatches + Permute
// (IFFT.compute:48-78), i.e. out[m] = (-1)^(mx+my) sum in[x,y] e^{+2 pi i (x mx + y my)/N}.
// Here one launch per direction replaces log2N launches: each workgroup holds
// whole length-N sequences in LDS and runs a Stockham autosort FFT with
// radix-16 stages (radix 2/4/8 for the last stage when log2N % 4 != 0), the
// butterflies in registers (64-lane waves, 16 complex values per lane), so
// every sequence crosses HBM once per direction (2 x 8 B read+write per texel).
//
// Stockham stage (radix R, Ns = product of earlier radices), for butterfly j:
//   v[r] = a[j + r N/R]; v[r] *= w_N^(r (j mod Ns) N/(Ns R)); V = IDFT_R(v);
//   b[(j / Ns) Ns R + (j mod Ns) + q Ns] = V[q]
// Twiddles come from a per-context table tw[m] = exp(+2 pi i m / N) built on
// the host in double precision (correctly rounded fp32).
//
// LDS layout: element i of the workgroup's tile at lds[i + (i >> 4)] (one
// complex of padding per 16) so the stride-R Stockham writes spread over banks.
//
// Kernels
//   k_rows<N>        in-place row pass (x direction) over one plane of every unit
//   k_cols<N>        in-place column pass (y direction) + (-1)^(x+y) permute
//   k_pass_a<N, P>   fused: evolve (TimeDependentSpectrum.compute:20-47) of the
//                    P planes of one row -> LDS -> row IFFT -> planes
//   k_pass_b<N, P>   fused: column IFFT of every plane of a W-column tile, permute,
//                    then FillResultTextures (ResultTexturesFiller.compute:16-34)
//                    in registers: DISP, DERIV, TURB (foam), NORMAL
#include "ocean_internal.h"
#include "spectrum_math.h"
#include "fft_core.h"

namespace ocean {
namespace {
using namespace fftcore;

// Sequence/butterfly bookkeeping.  A workgroup transforms B sequences of
// length N with THREADS = B*N/16 lanes.  Butterfly g = tid + m*THREADS of
// stage s maps to (sequence b, butterfly j) either j-fastest (rows: a lane
// group walks one contiguous sequence) or b-fastest (column tiles: a lane
// group walks the W columns of one row).
template <int N, int B, bool SEQ_FAST>
struct Map {
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
    // LDS index of element y of sequence b
    static __device__ __forceinline__ int lidx(int b, int y) {
        if constexpr (SEQ_FAST) return pad(y * B + b);
        else return pad(b * N + y);
    }
};

// Middle/last stages.  Stage S reads its inputs from LDS; if S is the last
// stage the outputs go to `store(b, y, value, m, q)`, else back to LDS.
template <int N, int B, bool SEQ_FAST, int S, class Store>
__device__ __forceinline__ void run_stages_from(float2* lds, const float2* __restrict__ tw, Store& store) {
    constexpr int R = radix_of(N, S);
    constexpr int NS = ns_of(N, S);
    constexpr int THREADS = B * N / kElems;
    constexpr int BF = kElems / R;  // butterflies per lane
    constexpr bool LAST = (S == n_stages(N) - 1);
    using M = Map<N, B, SEQ_FAST>;
    const int tid = threadIdx.x;
    float2 v[BF][R];
#pragma unroll
    for (int m = 0; m < BF; ++m) {
        int b, j;
        M::template bj<R>(tid + m * THREADS, b, j);
#pragma unroll
        for (int r = 0; r < R; ++r) v[m][r] = lds[M::lidx(b, j + r * (N / R))];
    }
    if constexpr (!LAST) __syncthreads();
#pragma unroll
    for (int m = 0; m < BF; ++m) {
        int b, j;
        M::template bj<R>(tid + m * THREADS, b, j);
        butterfly<N, R, NS>(v[m], j, tw);
        const int base = (j / NS) * NS * R + (j & (NS - 1));
#pragma unroll
        for (int q = 0; q < R; ++q) {
            if constexpr (LAST) store(b, base + q * NS, v[m][q], m, q);
            else lds[M::lidx(b, base + q * NS)] = v[m][q];
        }
    }
    if constexpr (!LAST) {
        __syncthreads();
        run_stages_from<N, B, SEQ_FAST, S + 1>(lds, tw, store);
    }
}

// Full transform: stage 0 reads `load(b, y)` (global memory or LDS), the
// last stage hands results to `store`.  If FROM_LDS, stage 0's inputs are in
// LDS already (a barrier separates their reads from the in-place writes).
template <int N, int B, bool SEQ_FAST, bool FROM_LDS, class Load, class Store>
__device__ __forceinline__ void lds_fft(float2* lds, const float2* __restrict__ tw, Load& load, Store& store) {
    if constexpr (FROM_LDS) {
        run_stages_from<N, B, SEQ_FAST, 0>(lds, tw, store);
    } else {
        constexpr int R = radix_of(N, 0);
        constexpr int THREADS = B * N / kElems;
        constexpr int BF = kElems / R;
        constexpr bool LAST = (n_stages(N) == 1);
        using M = Map<N, B, SEQ_FAST>;
        const int tid = threadIdx.x;
        float2 v[BF][R];
#pragma unroll
        for (int m = 0; m < BF; ++m) {
            int b, j;
            M::template bj<R>(tid + m * THREADS, b, j);
#pragma unroll
            for (int r = 0; r < R; ++r) v[m][r] = load(b, j + r * (N / R));
        }
#pragma unroll
        for (int m = 0; m < BF; ++m) {
            int b, j;
            M::template bj<R>(tid + m * THREADS, b, j);
            Idft<R>::run(v[m]);  // stage 0: Ns = 1, no twiddles
            const int base = j * R;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                if constexpr (LAST) store(b, base + q, v[m][q], m, q);
                else lds[M::lidx(b, base + q)] = v[m][q];
            }
        }
        if constexpr (!LAST) {
            __syncthreads();
            run_stages_from<N, B, SEQ_FAST, 1>(lds, tw, store);
        }
    }
}

// ------------------------------- kernels ---------------------------------

// Row pass: B = rows per workgroup (consecutive rows of the flattened
// [unit][y] row list of one plane).  In place.
template <int N>
constexpr int rows_per_wg() { return N >= 1024 ? 4 : 4096 / N; }

template <int N>
__global__ __launch_bounds__(rows_per_wg<N>() * N / kElems) void k_rows(float2* __restrict__ plane, int total_rows,
                                                                         const float2* __restrict__ tw) {
    constexpr int B = rows_per_wg<N>();
    __shared__ float2 lds[padded(B * N)];
    const int row0 = blockIdx.x * B;
    auto load = [&](int b, int x) -> float2 {
        const int row = row0 + b;
        return row < total_rows ? plane[(size_t)row * N + x] : make_float2(0.f, 0.f);
    };
    auto store = [&](int b, int x, float2 val, int, int) {
        const int row = row0 + b;
        if (row < total_rows) plane[(size_t)row * N + x] = val;
    };
    lds_fft<N, B, false, false>(lds, tw, load, store);
}

// Column pass + Permute: one workgroup = W consecutive columns of one unit.
template <int N>
__global__ __launch_bounds__(col_tile(N) * N / kElems) void k_cols(float2* __restrict__ plane,
                                                                   const float2* __restrict__ tw) {
    constexpr int W = col_tile(N);
    __shared__ float2 lds[padded(W * N)];
    constexpr int tiles = N / W;
    const int u = blockIdx.x / tiles;
    const int x0 = (blockIdx.x - u * tiles) * W;
    float2* base = plane + (size_t)u * N * N + x0;
    auto load = [&](int b, int y) -> float2 { return base[(size_t)y * N + b]; };
    auto store = [&](int b, int y, float2 val, int, int) {
        const float sgn = ((x0 + b + y) & 1) ? -1.0f : 1.0f;  // IFFT.compute:76
        base[(size_t)y * N + b] = make_float2(val.x * sgn, val.y * sgn);
    };
    lds_fft<N, W, true, false>(lds, tw, load, store);
}

// Fused pass A: evolve + row IFFT.  A workgroup owns RB rows; sequence
// b = p * RB + row (P planes).  Evolve writes the LDS tile directly.
template <int N, int P>
constexpr int pa_rows() { return (N >= 1024) ? 1 : 1024 / N; }

template <int N, int P>
__global__ __launch_bounds__((pa_rows<N, P>() * P * N / kElems)) void k_pass_a(DevView v, float time, int total_rows) {
    constexpr int RB = pa_rows<N, P>();
    constexpr int B = RB * P;
    constexpr int THREADS = B * N / kElems;
    __shared__ float2 lds[padded(B * N)];
    using M = Map<N, B, false>;
    const int row0 = blockIdx.x * RB;
    // evolve: RB*N texels, THREADS lanes
    for (int e = threadIdx.x; e < RB * N; e += THREADS) {
        const int rr = e / N, x = e - rr * N;
        const int row = row0 + rr;
        Planes4 o;
        if (row < total_rows) {
            const size_t i = (size_t)row * N + x;
            o = evolve_texel(v.h0[i], v.waves[i], time);
        } else {
            o.p[0] = o.p[1] = o.p[2] = o.p[3] = make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int p = 0; p < P; ++p) lds[M::lidx(p * RB + rr, x)] = o.p[p];
    }
    __syncthreads();
    auto load = [&](int, int) -> float2 { return make_float2(0.f, 0.f); };  // unused (FROM_LDS)
    auto store = [&](int b, int x, float2 val, int, int) {
        const int p = b / RB, rr = b - p * RB;
        const int row = row0 + rr;
        if (row < total_rows) v.plane[p][(size_t)row * N + x] = val;
    };
    (void)load;
    run_stages_from<N, B, false, 0>(lds, v.tw, store);
}

// Fused pass B: column IFFT of each plane of a W-column tile of one unit,
// permute, then the filler epilogue in registers.  Plane order 1, 0, 2, 3 keeps
// at most Dxz + (Dyx, Dyz) live per texel across planes.
template <int N, int P>
__global__ __launch_bounds__(col_tile(N) * N / kElems) void k_pass_b(DevView v) {
    constexpr int W = col_tile(N);
    constexpr int SL = n_stages(N) - 1;
    constexpr int RL = radix_of(N, SL);
    constexpr int BF = kElems / RL;
    __shared__ float2 lds[padded(W * N)];
    constexpr int tiles = N / W;
    const int u = blockIdx.x / tiles;
    const int x0 = (blockIdx.x - u * tiles) * W;
    const size_t ubase = (size_t)u * N * N + x0;

    float keep_a[BF][RL];  // plane 1: Dy, later Dxz
    float keep_b[BF][RL];  // plane 1: Dxz
    float keep_c[BF][RL];  // plane 2: Dyx
    float keep_d[BF][RL];  // plane 2: Dyz

    // ---- plane 1 (DyDxz): keep Dy and Dxz
    {
        const float2* src = v.plane[1] + ubase;
        auto load = [&](int b, int y) -> float2 { return src[(size_t)y * N + b]; };
        auto store = [&](int b, int y, float2 val, int m, int q) {
            const float sgn = ((x0 + b + y) & 1) ? -1.0f : 1.0f;
            keep_a[m][q] = val.x * sgn;
            keep_b[m][q] = val.y * sgn;
        };
        lds_fft<N, W, true, false>(lds, v.tw, load, store);
    }
    __syncthreads();
    // ---- plane 0 (DxDz): write DISP = (Dx, Dy, Dz, 1)
    {
        const float2* src = v.plane[0] + ubase;
        auto load = [&](int b, int y) -> float2 { return src[(size_t)y * N + b]; };
        auto store = [&](int b, int y, float2 val, int m, int q) {
            const float sgn = ((x0 + b + y) & 1) ? -1.0f : 1.0f;
            v.disp[ubase + (size_t)y * N + b] = make_float4(val.x * sgn, keep_a[m][q], val.y * sgn, 1.0f);
        };
        lds_fft<N, W, true, false>(lds, v.tw, load, store);
    }
    if constexpr (P == 4) {
        __syncthreads();
        // ---- plane 2 (DyxDyz): keep
        {
            const float2* src = v.plane[2] + ubase;
            auto load = [&](int b, int y) -> float2 { return src[(size_t)y * N + b]; };
            auto store = [&](int b, int y, float2 val, int m, int q) {
                const float sgn = ((x0 + b + y) & 1) ? -1.0f : 1.0f;
                keep_c[m][q] = val.x * sgn;
                keep_d[m][q] = val.y * sgn;
            };
            lds_fft<N, W, true, false>(lds, v.tw, load, store);
        }
        __syncthreads();
        // ---- plane 3 (DxxDzz): DERIV, Jacobian -> foam (TURB), NORMAL
        {
            const float2* src = v.plane[3] + ubase;
            auto load = [&](int b, int y) -> float2 { return src[(size_t)y * N + b]; };
            auto store = [&](int b, int y, float2 val, int m, int q) {
                const float sgn = ((x0 + b + y) & 1) ? -1.0f : 1.0f;
                const float dxx = val.x * sgn, dzz = val.y * sgn;
                const size_t i = ubase + (size_t)y * N + b;
                const float dyx = keep_c[m][q], dyz = keep_d[m][q];
                v.deriv[i] = make_float4(dyx, dyz, dxx, dzz);
                const float foam = foam_update(v.turb[i].x, dxx, dzz, keep_b[m][q]);
                v.turb[i] = make_float4(foam, foam, foam, foam);
                if (v.normals) v.normal[i] = normal_from_deriv(dyx, dyz, dxx, dzz);
            };
            lds_fft<N, W, true, false>(lds, v.tw, load, store);
        }
    }
}

// ------------------------------ dispatch ---------------------------------
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
struct RowsL {
    static hipError_t go(const DevView* v, int p, hipStream_t s) {
        constexpr int B = rows_per_wg<N>();
        const int total = v->units * N;
        hipLaunchKernelGGL(k_rows<N>, dim3((total + B - 1) / B), dim3(B * N / kElems), 0, s, v->plane[p], total, v->tw);
        return hipGetLastError();
    }
};
template <int N>
struct ColsL {
    static hipError_t go(const DevView* v, int p, hipStream_t s) {
        constexpr int W = col_tile(N);
        hipLaunchKernelGGL(k_cols<N>, dim3(v->units * (N / W)), dim3(W * N / kElems), 0, s, v->plane[p], v->tw);
        return hipGetLastError();
    }
};
template <int N>
struct PassAL {
    static hipError_t go(const DevView* v, float t, hipStream_t s) {
        const int total = v->units * N;
        if (v->planes == 4) {
            constexpr int RB = pa_rows<N, 4>();
            hipLaunchKernelGGL((k_pass_a<N, 4>), dim3((total + RB - 1) / RB), dim3(RB * 4 * N / kElems), 0, s, *v, t,
                               total);
        } else {
            constexpr int RB = pa_rows<N, 2>();
            hipLaunchKernelGGL((k_pass_a<N, 2>), dim3((total + RB - 1) / RB), dim3(RB * 2 * N / kElems), 0, s, *v, t,
                               total);
        }
        return hipGetLastError();
    }
};
template <int N>
struct PassBL {
    static hipError_t go(const DevView* v, hipStream_t s) {
        constexpr int W = col_tile(N);
        if (v->planes == 4)
            hipLaunchKernelGGL((k_pass_b<N, 4>), dim3(v->units * (N / W)), dim3(W * N / kElems), 0, s, *v);
        else
            hipLaunchKernelGGL((k_pass_b<N, 2>), dim3(v->units * (N / W)), dim3(W * N / kElems), 0, s, *v);
        return hipGetLastError();
    }
};

}  // namespace

hipError_t launch_ifft_rows(const DevView& v, int p, hipStream_t s) { return dispatch_n<RowsL>(v.n, &v, p, s); }
hipError_t launch_ifft_cols(const DevView& v, int p, hipStream_t s) { return dispatch_n<ColsL>(v.n, &v, p, s); }
hipError_t launch_pass_a(const DevView& v, float t, hipStream_t s) { return dispatch_n<PassAL>(v.n, &v, t, s); }
hipError_t launch_pass_b(const DevView& v, hipStream_t s) { return dispatch_n<PassBL>(v.n, &v, s); }

}  // namespace ocean
