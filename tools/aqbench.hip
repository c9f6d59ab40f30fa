// Pass AQ's memory shape without the evolve and the FFT: per item (unit,
// mirror-pair rows y1 = i, y2 = N - i) h0k of both rows is read (8 B per texel) and three planes of
// both rows are written into the 8-wide tile-major intermediate [plane][unit][x / 8][y][8] (24 B per
// texel), 4 x 1024^2 texels: 134 MB per launch, 3 workgroups of 256 lanes per CU as pass AQ.
//   0: pass AQ's rows (y1, N - y1): every store instruction writes 64-byte tile rows, the other
//      half of each 128-byte line comes from another item
//   1: rows (2i, 2i + 1): lanes 0-7 / 8-15 of each 16 write rows y, y + 1 of one tile, whole lines
//   2: the same bytes as flat contiguous streams (grid-stride)
// Build: hipcc --offload-arch=gfx950 -O3 tools/aqbench.hip -o tools/aqbench
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

constexpr int N = 1024, W = 8, T = 256;

template <int MODE>
__global__ __launch_bounds__(T) void k_aq_mem(const float2* __restrict__ h0k, float2* __restrict__ inter, size_t ps,
                                              int items_per_unit, int items) {
    const int l = threadIdx.x;
    for (int item = blockIdx.x; item < items; item += gridDim.x) {
        const int u = item / items_per_unit, i = item % items_per_unit;
        const int y1 = MODE == 1 ? 2 * i : i, y2 = MODE == 1 ? 2 * i + 1 : (i ? N - i : N / 2);
        float2 a[4], b[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            a[r] = h0k[((size_t)u * N + y1) * N + l + r * T];
            b[r] = h0k[((size_t)u * N + y2) * N + ((N - l - r * T) & (N - 1))];
        }
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float2 va = make_float2(a[q].x * (p + 1), b[q].y), vb = make_float2(b[q].x, a[q].y * (p + 2));
                float2* pl = inter + p * ps + (size_t)u * N * N;
                if (MODE == 1) {
                    // 16-lane group g covers tile 2 g' of the quarter: lanes 0-7 row y1, 8-15 row y2
                    const int g = l >> 4, s = (l >> 3) & 1, c = l & 7;
                    const int x = (g + 16 * q) * W + c;  // tiles g + 16 q, 64 tiles per q-pass... x < N
                    const float2 v0 = s ? vb : va;
                    pl[(size_t)(x / W) * N * W + (size_t)(s ? y2 : y1) * W + c] = v0;
                    const int x2 = x + 512;
                    pl[(size_t)(x2 / W) * N * W + (size_t)(s ? y1 : y2) * W + c] = s ? va : vb;
                } else {
                    const int x = l + q * T;
                    pl[(size_t)(x / W) * N * W + (size_t)y1 * W + x % W] = va;
                    pl[(size_t)(x / W) * N * W + (size_t)y2 * W + x % W] = vb;
                }
            }
    }
}

__global__ void k_flat(const float2* __restrict__ h0k, float2* __restrict__ inter, size_t ps, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float2 a = h0k[i];
        inter[i] = a;
        inter[ps + i] = make_float2(a.y, a.x);
        inter[2 * ps + i] = make_float2(-a.x, a.y);
    }
}

int main() {
    const int units = 4;
    const size_t tex = (size_t)units * N * N;
    float2 *h0k, *inter;
    CK(hipMalloc(&h0k, tex * 8));
    CK(hipMalloc(&inter, tex * 24));
    CK(hipMemset(h0k, 0, tex * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const double bytes = (double)tex * 32;
    for (int mode = 0; mode < 3; ++mode) {
        // mode 0: N/2 + 1 items per unit (row pairs, rows 0 and N/2 together); mode 1: N/2 row pairs
        const int ipu = mode == 0 ? N / 2 + 1 : N / 2;
        const int items = units * ipu;
        auto run = [&]() {
            if (mode == 0) hipLaunchKernelGGL(k_aq_mem<0>, dim3(768), dim3(T), 0, 0, h0k, inter, tex, ipu, items);
            if (mode == 1) hipLaunchKernelGGL(k_aq_mem<1>, dim3(768), dim3(T), 0, 0, h0k, inter, tex, ipu, items);
            if (mode == 2) hipLaunchKernelGGL(k_flat, dim3(4096), dim3(256), 0, 0, h0k, inter, tex, tex);
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
        const char* names[] = {"AQ rows (y, N - y), half lines", "rows (y, y + 1), whole lines", "flat streams"};
        printf("%-34s %8.1f us %8.1f GB/s\n", names[mode], us, bytes / us / 1e3);
    }
    return 0;
}
