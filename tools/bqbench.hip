// Pass BQ's memory shape without the FFT ("What holds each hot kernel"; docs/MEASUREMENTS.md section 3): per item
// (unit, 8-column tile) three 64 KiB tile-major plane blocks are read (24 B per texel), the foam
// state read and written (4 + 4 B), and three float4 textures written (48 B), 4 x 1024^2 texels:
// 335 MB per launch.  Variants of the texture stores only:
//   0: texture layout [u][y][x], 128 B per row per tile, nontemporal (pass BQ)
//   1: the same, default policy
//   2: tile-major outputs [u][tile][y][8] (contiguous 128 KiB per tile and texture), nontemporal:
//      the write-locality bound the texture layout gives up
//   3: texture layout, rows written in the order q-major across the workgroup's lanes (each store
//      instruction of a wave covers 8 consecutive rows, as 0, but the workgroup sweeps the tile
//      top to bottom: rows 8w + 64 i -> 512 i + 8 w)
//   4: as 0 without the foam state (72 B per texel)
//   5: as 4 with 16-B plane loads (k_bq_mem16; its two half-line stores per lane dominate)
//   6: as 4 as flat contiguous streams (k_flat)
//   7: as 6 with Q1 and Q2 interleaved into one 16-byte read stream (k_flat2)
//   8: as 0's 80 B (foam state included) as flat contiguous streams (k_flat_foam): whole-line stores
//      everywhere at pass BQ's own byte count, the bound a row-contiguous (column-first) pass B could reach
//   9: as 0 with the foam state read back from TURB.x (a 16-B read) and no separate foam array (88 B)
//  10: as 0 with the foam state written by nontemporal stores
//  11: as 0 with the foam loads issued first (before the plane loads) and the foam stores last
//  12: as 0 with TURB carrying the new foam (the texture depends on the foam read, as in pass BQ)
//  13: as 12 with the first texture (DISP) written by default-policy stores and the plane loads nontemporal:
//      pass BQ's DC form (the frame's re-read set plus DISP in the Infinity Cache)
//  14: as 12 with the foam state lane-major (each lane's 16 values contiguous: 4 float4 loads and stores
//      instead of 16 + 16 dword accesses)
// Build: hipcc --offload-arch=gfx950 -O3 tools/bqbench.hip -o tools/bqbench
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int N = 1024, W = 8, TILE = W * N, T = 512;

// 5: as 4 (no foam) with 16-B plane loads (a lane holds two adjacent columns, half the rows)
__global__ __launch_bounds__(T) void k_bq_mem16(const f32x4* __restrict__ tp, size_t ps4, f32x4* __restrict__ d0,
                                                f32x4* __restrict__ d1, f32x4* __restrict__ d2, int items) {
    const int lb2 = threadIdx.x % (W / 2), lj = threadIdx.x / (W / 2);  // lj < 128
    f32x4 v[3][8];
    for (int item = blockIdx.x; item < items; item += gridDim.x) {
        const int u = item / (N / W), x0 = (item % (N / W)) * W;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const f32x4* src = tp + p * ps4 + (size_t)item * (TILE / 2) + lj * (W / 2) + lb2;
#pragma unroll
            for (int i = 0; i < 8; ++i) v[p][i] = src[i * 128 * (W / 2)];
        }
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            f32x4* dst = t == 0 ? d0 : (t == 1 ? d1 : d2);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const f32x4 a = v[t][i], b = v[(t + 1) % 3][i];
                const f32x4 v0 = {a.x, b.y, a.y, 1.0f}, v1 = {a.z, b.w, a.w, 1.0f};
                f32x4* o = dst + (size_t)u * N * N + (size_t)(lj + i * 128) * N + x0 + 2 * lb2;
                __builtin_nontemporal_store(v0, o);
                __builtin_nontemporal_store(v1, o + 1);
            }
        }
    }
}

// 6: the same bytes as 4 (three float2 plane reads, three float4 texture writes per texel) as a
// flat grid-stride stream over texels: no tiles, every access contiguous across the wave
__global__ void k_flat(const float2* __restrict__ tp, size_t ps, f32x4* __restrict__ d0, f32x4* __restrict__ d1,
                       f32x4* __restrict__ d2, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float2 a = tp[i], b = tp[ps + i], c = tp[2 * ps + i];
        const f32x4 v0 = {a.x, b.y, a.y, 1.0f}, v1 = {b.x, c.y, b.y, 1.0f}, v2 = {c.x, a.y, c.y, 1.0f};
        __builtin_nontemporal_store(v0, d0 + i);
        __builtin_nontemporal_store(v1, d1 + i);
        __builtin_nontemporal_store(v2, d2 + i);
    }
}

// 7: as 6 with Q1, Q2 interleaved (one 16-byte read stream) and Q3 apart (8 bytes)
__global__ void k_flat2(const f32x4* __restrict__ q12, const float2* __restrict__ q3, f32x4* __restrict__ d0,
                        f32x4* __restrict__ d1, f32x4* __restrict__ d2, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const f32x4 ab = q12[i];
        const float2 c = q3[i];
        const f32x4 v0 = {ab.x, ab.w, ab.y, 1.0f}, v1 = {ab.z, c.y, ab.w, 1.0f}, v2 = {c.x, ab.y, c.y, 1.0f};
        __builtin_nontemporal_store(v0, d0 + i);
        __builtin_nontemporal_store(v1, d1 + i);
        __builtin_nontemporal_store(v2, d2 + i);
    }
}

// 8: the bytes of 0 (planes, foam state read + write, three textures) as flat streams
__global__ void k_flat_foam(const float2* __restrict__ tp, size_t ps, float* __restrict__ foam, f32x4* __restrict__ d0,
                            f32x4* __restrict__ d1, f32x4* __restrict__ d2, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float2 a = tp[i], b = tp[ps + i], c = tp[2 * ps + i];
        const float f = foam[i] * 0.5f + c.x;
        foam[i] = f;
        const f32x4 v0 = {a.x, b.y, a.y, 1.0f}, v1 = {b.x, c.y, f, 1.0f}, v2 = {c.x, a.y, c.y, f};
        __builtin_nontemporal_store(v0, d0 + i);
        __builtin_nontemporal_store(v1, d1 + i);
        __builtin_nontemporal_store(v2, d2 + i);
    }
}

template <int MODE>
__global__ __launch_bounds__(T) void k_bq_mem(const float2* __restrict__ tp, size_t ps, float* __restrict__ foam,
                                              f32x4* __restrict__ d0, f32x4* __restrict__ d1, f32x4* __restrict__ d2,
                                              int items) {
    const int lb = threadIdx.x % W, lj = threadIdx.x / W;  // lj < 64
    float2 v[3][16];
    for (int item = blockIdx.x; item < items; item += gridDim.x) {
        const int u = item / (N / W), x0 = (item % (N / W)) * W;
        float fl[16];
        float* fp = foam + (size_t)item * TILE + lj * W + lb;
        if (MODE == 11) {
#pragma unroll
            for (int i = 0; i < 16; ++i) fl[i] = fp[i * 64 * W];
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const float2* src = tp + p * ps + (size_t)item * TILE + lj * W + lb;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if (MODE == 13) {
                    typedef float f32x2 __attribute__((ext_vector_type(2)));
                    const f32x2 x = __builtin_nontemporal_load(reinterpret_cast<const f32x2*>(src + i * 64 * W));
                    v[p][i] = make_float2(x.x, x.y);
                } else {
                    v[p][i] = src[i * 64 * W];
                }
            }
        }
        float fs[16];
        if (MODE == 14) {
            const int lane = lj * W + lb;
            const f32x4* f4 = reinterpret_cast<const f32x4*>(foam + (size_t)item * TILE) + lane * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const f32x4 x = f4[k];
                fs[4 * k] = x.x * 0.5f + v[2][4 * k].x;
                fs[4 * k + 1] = x.y * 0.5f + v[2][4 * k + 1].x;
                fs[4 * k + 2] = x.z * 0.5f + v[2][4 * k + 2].x;
                fs[4 * k + 3] = x.w * 0.5f + v[2][4 * k + 3].x;
            }
        } else if (MODE == 9) {  // the foam state is TURB.x of the previous frame (d2 plays TURB)
#pragma unroll
            for (int i = 0; i < 16; ++i)
                fs[i] = d2[(size_t)u * N * N + (size_t)(lj + i * 64) * N + x0 + lb].x * 0.5f + v[2][i].x;
        } else if (MODE == 10) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                fs[i] = fp[i * 64 * W] * 0.5f + v[2][i].x;
                __builtin_nontemporal_store(fs[i], fp + i * 64 * W);
            }
        } else if (MODE == 11) {
#pragma unroll
            for (int i = 0; i < 16; ++i) fs[i] = fl[i] * 0.5f + v[2][i].x;
        } else if (MODE != 4) {
#pragma unroll
            for (int i = 0; i < 16; ++i) fp[i * 64 * W] = fs[i] = fp[i * 64 * W] * 0.5f + v[2][i].x;
        }
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            f32x4* dst = t == 0 ? d0 : (t == 1 ? d1 : d2);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const f32x4 val = {(MODE == 9 || MODE >= 12) && t == 2 ? fs[i] : v[t][i].x, v[(t + 1) % 3][i].y,
                                   v[t][i].y, 1.0f};
                size_t o;
                if (MODE == 2) {
                    o = (size_t)item * TILE + (size_t)(lj + i * 64) * W + lb;
                } else if (MODE == 3) {
                    const int w = lj >> 3, r = lj & 7;       // wave w, row r within its 8
                    const int yy = i * 64 + w * 8 + r;       // waves sweep consecutive 8-row blocks
                    o = (size_t)u * N * N + (size_t)yy * N + x0 + lb;
                } else {
                    o = (size_t)u * N * N + (size_t)(lj + i * 64) * N + x0 + lb;
                }
                if (MODE == 1 || (MODE == 13 && t == 0)) dst[o] = val;
                else __builtin_nontemporal_store(val, dst + o);
            }
        }
        if (MODE == 11) {
#pragma unroll
            for (int i = 0; i < 16; ++i) fp[i * 64 * W] = fs[i];
        }
        if (MODE == 14) {
            f32x4* f4 = reinterpret_cast<f32x4*>(foam + (size_t)item * TILE) + (lj * W + lb) * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const f32x4 x = {fs[4 * k], fs[4 * k + 1], fs[4 * k + 2], fs[4 * k + 3]};
                f4[k] = x;
            }
        }
    }
}

int main() {
    const int units = 4;
    const size_t tex = (size_t)units * N * N;
    float2* tp;
    float* foam;
    f32x4 *d0, *d1, *d2;
    CK(hipMalloc(&tp, tex * 8 * 3));
    CK(hipMalloc(&foam, tex * 4));
    CK(hipMalloc(&d0, tex * 16));
    CK(hipMalloc(&d1, tex * 16));
    CK(hipMalloc(&d2, tex * 16));
    CK(hipMemset(tp, 0, tex * 24));
    CK(hipMemset(foam, 0, tex * 4));
    const int items = units * (N / W);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const double bytes_all = (double)tex * (24 + 8 + 48);
    for (int grid : {256, 512}) {
        printf("grid %d (%d workgroups of %d lanes per CU)\n", grid, grid / 256, T);
        for (int mode = 0; mode < 15; ++mode) {
            auto run = [&]() {
                if (mode == 0) hipLaunchKernelGGL(k_bq_mem<0>, dim3(grid), dim3(T), 0, 0, tp, tex, foam, d0, d1, d2, items);
                if (mode == 1) hipLaunchKernelGGL(k_bq_mem<1>, dim3(grid), dim3(T), 0, 0, tp, tex, foam, d0, d1, d2, items);
                if (mode == 2) hipLaunchKernelGGL(k_bq_mem<2>, dim3(grid), dim3(T), 0, 0, tp, tex, foam, d0, d1, d2, items);
                if (mode == 3) hipLaunchKernelGGL(k_bq_mem<3>, dim3(grid), dim3(T), 0, 0, tp, tex, foam, d0, d1, d2, items);
                if (mode == 4) hipLaunchKernelGGL(k_bq_mem<4>, dim3(grid), dim3(T), 0, 0, tp, tex, foam, d0, d1, d2, items);
                if (mode == 5)
                    hipLaunchKernelGGL(k_bq_mem16, dim3(grid), dim3(T), 0, 0, (const f32x4*)tp, tex / 2, d0, d1, d2, items);
                if (mode == 6) hipLaunchKernelGGL(k_flat, dim3(grid * 8), dim3(256), 0, 0, tp, tex, d0, d1, d2, tex);
                if (mode == 8) hipLaunchKernelGGL(k_flat_foam, dim3(grid * 8), dim3(256), 0, 0, tp, tex, foam, d0, d1, d2, tex);
                if (mode == 9) hipLaunchKernelGGL(k_bq_mem<9>, dim3(grid), dim3(T), 0, 0, tp, tex, foam, d0, d1, d2, items);
                if (mode == 10) hipLaunchKernelGGL(k_bq_mem<10>, dim3(grid), dim3(T), 0, 0, tp, tex, foam, d0, d1, d2, items);
                if (mode == 11) hipLaunchKernelGGL(k_bq_mem<11>, dim3(grid), dim3(T), 0, 0, tp, tex, foam, d0, d1, d2, items);
                if (mode == 12) hipLaunchKernelGGL(k_bq_mem<12>, dim3(grid), dim3(T), 0, 0, tp, tex, foam, d0, d1, d2, items);
                if (mode == 13) hipLaunchKernelGGL(k_bq_mem<13>, dim3(grid), dim3(T), 0, 0, tp, tex, foam, d0, d1, d2, items);
                if (mode == 14) hipLaunchKernelGGL(k_bq_mem<14>, dim3(grid), dim3(T), 0, 0, tp, tex, foam, d0, d1, d2, items);
                if (mode == 7)
                    hipLaunchKernelGGL(k_flat2, dim3(grid * 8), dim3(256), 0, 0, (const f32x4*)tp, tp + 2 * tex, d0, d1, d2,
                                       tex);
            };
            for (int w = 0; w < 3; ++w) run();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int r = 0; r < 50; ++r) run();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const double us = ms * 1e3 / 50;
            const char* names[] = {"texture layout, nt", "texture layout, plain", "tile-major outputs, nt",
                                   "texture layout, waves sweep rows", "texture layout, nt, no foam (-8 B)",
                                   "no foam, 16-B plane loads", "no foam, flat streams (grid x 8 WGs)",
                                   "no foam, flat, Q1|Q2 interleaved", "flat streams with foam (80 B)",
                                   "foam state from TURB.x (88 B)", "foam stores nontemporal",
                                   "foam loads first, stores last", "TURB carries the new foam",
                                   "as 12, DISP cached, nt plane loads", "as 12, foam lane-major (float4)"};
            const double bytes = (mode >= 4 && mode <= 7) ? bytes_all * 72 / 80 : (mode == 9 ? bytes_all * 88 / 80 : bytes_all);
            printf("%-34s %8.1f us %8.1f GB/s\n", names[mode], us, bytes / us / 1e3);
        }
    }
    return 0;
}
