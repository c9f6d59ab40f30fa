// Memory-pattern microbenchmark for the ocean path's access shapes on MI355X.
// Build: hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o tools/membench
// Each test moves a fixed byte count; prints GB/s (bytes read + written / time).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

constexpr int N = 1024;

// 1. streaming float4 copy (grid-stride)
__global__ void k_copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// 2. column-tile read of float2 planes: tile = W columns x N rows, lane (b = tid % W, j = tid / W)
//    reads rows j + 64 r (16 values), writes the same texels (in-place style copy to b)
template <int W>
__global__ void k_coltile(const float2* __restrict__ a, float2* __restrict__ b, int tiles_per_unit) {
    constexpr int T = W * N / 16;
    const int tile = blockIdx.x;
    const int u = tile / tiles_per_unit, x0 = (tile % tiles_per_unit) * W;
    const int lb = threadIdx.x % W, lj = threadIdx.x / W;
    const float2* src = a + (size_t)u * N * N + x0 + lb;
    float2* dst = b + (size_t)u * N * N + x0 + lb;
    constexpr int RS = T / W;  // rows between a lane's values
    float2 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = src[(size_t)(lj + r * RS) * N];
#pragma unroll
    for (int r = 0; r < 16; ++r) dst[(size_t)(lj + r * RS) * N] = v[r];
}

// 3. column-tile float4 stores (the pass-B epilogue shape): 16 B per lane, W texels per row
template <int W>
__global__ void k_coltile_store4(float4* __restrict__ b, int tiles_per_unit) {
    constexpr int T = W * N / 16;
    const int tile = blockIdx.x;
    const int u = tile / tiles_per_unit, x0 = (tile % tiles_per_unit) * W;
    const int lb = threadIdx.x % W, lj = threadIdx.x / W;
    float4* dst = b + (size_t)u * N * N + x0 + lb;
    constexpr int RS = T / W;
#pragma unroll
    for (int r = 0; r < 16; ++r) dst[(size_t)(lj + r * RS) * N] = make_float4(r, lj, lb, 1.f);
}

// 4. row read of float2 (the row pass shape): 4 rows per WG, lane reads j + 64 r
__global__ void k_rowtile(const float2* __restrict__ a, float2* __restrict__ b) {
    const size_t row0 = (size_t)blockIdx.x * 4;
    const int rb = threadIdx.x / 64, j = threadIdx.x % 64;
    const float2* src = a + (row0 + rb) * N + j;
    float2* dst = b + (row0 + rb) * N + j;
    float2 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = src[r * 64];
#pragma unroll
    for (int r = 0; r < 16; ++r) dst[r * 64] = v[r];
}

// 5. pass-A write shape: one row x 4 planes per 256-lane WG, wave = plane,
//    lane jj writes x = jj + 64 q.  MODE 0: tile-major [x/8][y][8] float2;
//    1: row-major float2; 2: tile-major, lane pairs as float4 (x even);
//    3: tile-major with two rows per WG (rows y, y+1 -> 128 B lines whole).
template <int MODE>
__global__ void k_wr_a(float2* __restrict__ t, size_t plane_stride, int rows) {
    const int p = threadIdx.x / 64, jj = threadIdx.x % 64;
    if (MODE == 3) {
        for (int row = blockIdx.x * 2; row < rows; row += gridDim.x * 2) {
            const int u = row / N, y = row % N;
            float2* base = t + p * plane_stride + (size_t)u * N * N + (size_t)y * 8;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                // lanes 0-7: row y cols 0-7 of tile, lanes 8-15 row y+1; 4 tiles per 16-lane group
                const int l = jj, r = (l >> 3) & 1, col = l & 7, tl = (l >> 4) + 4 * q;
                base[(size_t)tl * N * 8 + r * 8 + col] = make_float2(q, l);
                base[(size_t)(tl + 64) * N * 8 + r * 8 + col] = make_float2(q, -l);
            }
        }
        return;
    }
    for (int row = blockIdx.x; row < rows; row += gridDim.x) {
        const int u = row / N, y = row % N;
        float2* pl = t + p * plane_stride;
        if (MODE == 2) {
#pragma unroll
            for (int q = 0; q < 16; q += 2) {
                const int x = (jj & ~1) + (q + (jj & 1)) * 64;
                *(float4*)(pl + (size_t)u * N * N + (size_t)(x / 8) * N * 8 + y * 8 + x % 8) = make_float4(q, jj, 1, 2);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int x = jj + q * 64;
                const size_t o = MODE == 1 ? (size_t)row * N + x : (size_t)u * N * N + (size_t)(x / 8) * N * 8 + y * 8 + x % 8;
                pl[o] = make_float2(q, jj);
            }
        }
    }
}

// 6. pass-B memory shape without the FFT: item = (unit, 8-column tile); per
//    plane a contiguous 64 KiB tile read (next plane prefetched), then for three
//    planes a float4 texture tile write (8 columns x 1024 rows, 128-B rows) and
//    the compact foam read + write.  4 units: 369 MB per launch (88 B/texel).
template <int MODE>  // bit 1: no texture stores, 2: no foam, 4: no tile loads, 8: nontemporal stores
__global__ __launch_bounds__(512) void k_passb_mem(const float2* __restrict__ tp, size_t ps, float* __restrict__ foam,
                                                   float4* __restrict__ d0, float4* __restrict__ d1,
                                                   float4* __restrict__ d2, int items) {
    constexpr int W = 8, TILE = W * N;
    const int lb = threadIdx.x % W, lj = threadIdx.x / W;
    float2 cur[16], nxt[16];
    auto load = [&](int item, int p, float2* d) {
        const float2* src = tp + p * ps + (size_t)item * TILE + lj * W + lb;
#pragma unroll
        for (int i = 0; i < 16; ++i) d[i] = (MODE & 4) ? make_float2(i + item, p) : src[i * 64 * W];
    };
    int item = blockIdx.x;
    if (item < items) load(item, 0, cur);
    for (; item < items; item += gridDim.x) {
        const int u = item / (N / W), x0 = (item % (N / W)) * W;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            if (p < 3) load(item, p + 1, nxt);
            else if (item + (int)gridDim.x < items) load(item + gridDim.x, 0, nxt);
            float acc = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) acc += cur[i].x - cur[i].y;
            float4* dst = p == 0 ? d0 : (p == 2 ? d1 : d2);
            if (p == 3 && !(MODE & 2)) {
                float* f = foam + (size_t)item * TILE + lj * W + lb;
#pragma unroll
                for (int i = 0; i < 16; ++i) f[i * 64 * W] = f[i * 64 * W] * 0.5f + acc;
            }
            if (p != 1 && !(MODE & 1)) {
                float4* o = dst + (size_t)u * N * N + (size_t)lj * N + x0 + lb;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float4 val = make_float4(acc, cur[i].x, cur[i].y, 1.f);
                    if (MODE & 8) {
                        typedef float f4v __attribute__((ext_vector_type(4)));
                        f4v vv = {val.x, val.y, val.z, val.w};
                        __builtin_nontemporal_store(vv, reinterpret_cast<f4v*>(&o[(size_t)i * 64 * N]));
                    } else {
                        o[(size_t)i * 64 * N] = val;
                    }
                }
            } else if (MODE & 1) {
                if (acc == 12345.f) d0[threadIdx.x] = make_float4(acc, 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) cur[i] = nxt[i];
        }
    }
}

template <class F>
float timeit(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    const int units = 16;  // 16 x 1024^2 complex = 128 MiB per plane array (beyond L2, inside MALL)
    const size_t elems = (size_t)units * N * N;
    float2 *a, *b;
    float4* c;
    CK(hipMalloc(&a, elems * 8));
    CK(hipMalloc(&b, elems * 8));
    CK(hipMalloc(&c, elems * 16));
    CK(hipMemset(a, 0, elems * 8));
    CK(hipMemset(b, 0, elems * 8));
    CK(hipMemset(c, 0, elems * 16));
    const int reps = 20;
    {
        float ms = timeit([&] { hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, (const float4*)a, (float4*)b, elems / 2); }, reps);
        printf("copy float4            %8.1f GB/s  (%.1f us)\n", 2.0 * elems * 8 / ms / 1e6, ms * 1e3);
    }
    {
        float ms = timeit([&] { hipLaunchKernelGGL(k_rowtile, dim3(units * N / 4), dim3(256), 0, 0, a, b); }, reps);
        printf("row tile float2        %8.1f GB/s  (%.1f us)\n", 2.0 * elems * 8 / ms / 1e6, ms * 1e3);
    }
    {
        float ms = timeit([&] { hipLaunchKernelGGL(k_coltile<8>, dim3(units * N / 8), dim3(512), 0, 0, a, b, N / 8); }, reps);
        printf("col tile W=8 float2    %8.1f GB/s  (%.1f us)\n", 2.0 * elems * 8 / ms / 1e6, ms * 1e3);
    }
    {
        float ms = timeit([&] { hipLaunchKernelGGL(k_coltile<16>, dim3(units * N / 16), dim3(1024), 0, 0, a, b, N / 16); }, reps);
        printf("col tile W=16 float2   %8.1f GB/s  (%.1f us)\n", 2.0 * elems * 8 / ms / 1e6, ms * 1e3);
    }
    {
        float ms = timeit([&] { hipLaunchKernelGGL(k_coltile<4>, dim3(units * N / 4), dim3(256), 0, 0, a, b, N / 4); }, reps);
        printf("col tile W=4 float2    %8.1f GB/s  (%.1f us)\n", 2.0 * elems * 8 / ms / 1e6, ms * 1e3);
    }
    {
        float ms = timeit([&] { hipLaunchKernelGGL(k_coltile_store4<8>, dim3(units * N / 8), dim3(512), 0, 0, c, N / 8); }, reps);
        printf("col tile W=8 store f4  %8.1f GB/s  (%.1f us)\n", 1.0 * elems * 16 / ms / 1e6, ms * 1e3);
    }
    {
        float ms = timeit([&] { hipLaunchKernelGGL(k_coltile_store4<16>, dim3(units * N / 16), dim3(1024), 0, 0, c, N / 16); }, reps);
        printf("col tile W=16 store f4 %8.1f GB/s  (%.1f us)\n", 1.0 * elems * 16 / ms / 1e6, ms * 1e3);
    }
    {
        const int rows = 4 * N;  // 4 units (cfg3), 4 planes: 128 MiB written
        const size_t ps = (size_t)rows * N;
        const char* names[4] = {"passA tiled f2", "passA rowmajor f2", "passA tiled f4 pairs", "passA tiled 2 rows"};
        for (int mode = 0; mode < 4; ++mode)
            for (int grid : {768, 1024, 4096}) {
                auto f = [&] {
                    if (mode == 0) hipLaunchKernelGGL(k_wr_a<0>, dim3(grid), dim3(256), 0, 0, a, ps, rows);
                    if (mode == 1) hipLaunchKernelGGL(k_wr_a<1>, dim3(grid), dim3(256), 0, 0, a, ps, rows);
                    if (mode == 2) hipLaunchKernelGGL(k_wr_a<2>, dim3(grid), dim3(256), 0, 0, a, ps, rows);
                    if (mode == 3) hipLaunchKernelGGL(k_wr_a<3>, dim3(grid / 2), dim3(256), 0, 0, a, ps, rows);
                };
                float ms = timeit(f, reps);
                printf("%-22s grid %5d %8.1f GB/s  (%.1f us)\n", names[mode], grid, 4.0 * ps * 8 / ms / 1e6, ms * 1e3);
            }
    }
    {
        const int units4 = 4;
        const size_t ps = (size_t)units4 * N * N;
        float2* tp;
        float* fm;
        float4 *o0, *o1, *o2;
        CK(hipMalloc(&tp, ps * 8 * 4));
        CK(hipMalloc(&fm, ps * 4));
        CK(hipMalloc(&o0, ps * 16));
        CK(hipMalloc(&o1, ps * 16));
        CK(hipMalloc(&o2, ps * 16));
        CK(hipMemset(tp, 0, ps * 32));
        CK(hipMemset(fm, 0, ps * 4));
        const int items = units4 * (N / 8);
        auto run = [&](const char* name, auto kern, double bytes_per_texel) {
            for (int grid : {256, 512}) {
                float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, 0, tp, ps, fm, o0, o1, o2, items); }, reps);
                printf("passB %-22s grid %4d %8.1f GB/s  (%.1f us)\n", name, grid, bytes_per_texel * ps / ms / 1e6, ms * 1e3);
            }
        };
        run("full shape", k_passb_mem<0>, 88.0);
        run("no tex stores", k_passb_mem<1>, 40.0);
        run("no foam", k_passb_mem<2>, 80.0);
        run("no tile loads", k_passb_mem<4>, 56.0);
        run("stores only", k_passb_mem<6>, 48.0);
        run("nt stores", k_passb_mem<8>, 88.0);
    }
    return 0;
}
