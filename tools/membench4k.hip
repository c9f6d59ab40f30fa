// N = 4096 access shapes (cfg5): what the fused passes' memory traffic costs alone.
// Build: hipcc --offload-arch=gfx950 -O3 tools/membench4k.hip -o tools/membench4k
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 4096;
constexpr int U = 4;  // cascades

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

// pass-A write shape: WG = one row x 4 planes (1024 lanes), lane writes 16 float2.
// MODE 0: tile-major W=4 [x/4][y][4]; 1: row-major; 2: tile-major W=8; 3: W=16
template <int MODE>
__global__ __launch_bounds__(1024) void k_wr_a(float2* __restrict__ t, size_t ps, int rows) {
    constexpr int W = MODE == 2 ? 8 : (MODE == 3 ? 16 : 4);
    const int p = threadIdx.x / 256, jj = threadIdx.x % 256;
    const int g = gridDim.x;
    for (int item = (blockIdx.x % 8) * (g / 8) + blockIdx.x / 8; item < rows; item += g) {
        const int u = item / N, y = item % N;
        float2* pl = t + p * ps;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int x = jj + q * 256;
            const size_t o = MODE == 1 ? (size_t)item * N + x : (size_t)u * N * N + (size_t)(x / W) * N * W + (size_t)y * W + x % W;
            pl[o] = make_float2(q, jj);
        }
    }
}

// pass-B output shape: WG = W columns x N rows (tile), lane (b = tid % W, j = tid / W),
// 16 float4 stores per texture, 3 textures; tile reads 4 x (W*N*8) contiguous.
template <int W, bool READ>
__global__ __launch_bounds__(1024) void k_b_shape(const float2* __restrict__ tp, size_t ps, float4* __restrict__ o0,
                                                  float4* __restrict__ o1, float4* __restrict__ o2, int items) {
    constexpr int T = W * N / 16;
    const int lb = threadIdx.x % W, lj = threadIdx.x / W;
    for (int item = blockIdx.x; item < items; item += gridDim.x) {
        const int u = item / (N / W), x0 = (item % (N / W)) * W;
        float acc = 0.f;
        for (int p = 0; p < 4; ++p) {
            if (READ) {
                const float2* src = tp + p * ps + (size_t)item * W * N + lj * W + lb;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float2 v = src[(size_t)i * (T / W) * W];
                    acc += v.x - v.y;
                }
            }
            if (p == 1) continue;
            float4* dst = p == 0 ? o0 : (p == 2 ? o1 : o2);
            float4* o = dst + (size_t)u * N * N + (size_t)lj * N + x0 + lb;
#pragma unroll
            for (int i = 0; i < 16; ++i) o[(size_t)i * (T / W) * N] = make_float4(acc, i, p, 1.f);
        }
    }
}

int main() {
    const size_t ps = (size_t)U * N * N;
    float2* tp;
    float4 *o0, *o1, *o2;
    if (hipMalloc(&tp, ps * 32) != hipSuccess || hipMalloc(&o0, ps * 16) != hipSuccess ||
        hipMalloc(&o1, ps * 16) != hipSuccess || hipMalloc(&o2, ps * 16) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(tp, 0, ps * 32);
    const int reps = 5;
    const int rows = U * N;
    const char* an[4] = {"A write W=4 tile", "A write row-major", "A write W=8 tile", "A write W=16 tile"};
    for (int m = 0; m < 4; ++m) {
        auto f = [&] {
            if (m == 0) hipLaunchKernelGGL(k_wr_a<0>, dim3(256), dim3(1024), 0, 0, tp, ps, rows);
            if (m == 1) hipLaunchKernelGGL(k_wr_a<1>, dim3(256), dim3(1024), 0, 0, tp, ps, rows);
            if (m == 2) hipLaunchKernelGGL(k_wr_a<2>, dim3(256), dim3(1024), 0, 0, tp, ps, rows);
            if (m == 3) hipLaunchKernelGGL(k_wr_a<3>, dim3(256), dim3(1024), 0, 0, tp, ps, rows);
        };
        float ms = timeit(f, reps);
        printf("%-22s %8.1f GB/s (%.1f us)\n", an[m], 32.0 * ps / ms / 1e6, ms * 1e3);
    }
    {
        float ms = timeit([&] { hipLaunchKernelGGL((k_b_shape<4, true>), dim3(256), dim3(1024), 0, 0, tp, ps, o0, o1, o2, U * N / 4); }, reps);
        printf("B shape W=4 read+write %8.1f GB/s (%.1f us)\n", 80.0 * ps / ms / 1e6, ms * 1e3);
        ms = timeit([&] { hipLaunchKernelGGL((k_b_shape<4, false>), dim3(256), dim3(1024), 0, 0, tp, ps, o0, o1, o2, U * N / 4); }, reps);
        printf("B shape W=4 write only %8.1f GB/s (%.1f us)\n", 48.0 * ps / ms / 1e6, ms * 1e3);
        ms = timeit([&] { hipLaunchKernelGGL((k_b_shape<8, false>), dim3(512), dim3(1024), 0, 0, tp, ps, o0, o1, o2, U * N / 8); }, reps);
        printf("B shape W=8 write only %8.1f GB/s (%.1f us)\n", 48.0 * ps / ms / 1e6, ms * 1e3);
    }
    return 0;
}
