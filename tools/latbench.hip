// Launch-latency floor for small jobs (cfg2 analysis, docs/MEASUREMENTS.md section 6): the duration
// of back-to-back launches of (0) an empty kernel, (1) a kernel whose workgroups load one
// 16 KiB block each and (2) load it, wait, and store it back elsewhere -- 256 workgroups of
// 128 lanes, one item each, as pass A3 runs at cfg2.  Prints microseconds per launch.
//   hipcc --offload-arch=gfx950 -O3 -o tools/latbench tools/latbench.hip && tools/latbench
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(128) void k_empty(float* out) {
    if (threadIdx.x == 1024) out[0] = 0.0f;  // never true: keeps the kernel from being empty-bodied
}

__global__ __launch_bounds__(128) void k_load(const float4* in, float* out) {
    const float4* b = in + (size_t)blockIdx.x * 1024;
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float4 v = b[i * 128 + threadIdx.x];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.0f) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(128) void k_copy(const float4* in, float4* out) {
    const float4* b = in + (size_t)blockIdx.x * 1024;
    float4* o = out + (size_t)blockIdx.x * 1024;
    float4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = b[i * 128 + threadIdx.x];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i * 128 + threadIdx.x] = v[i];
}

int main() {
    const int blocks = 256, reps = 2000;
    float4 *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, (size_t)blocks * 1024 * 16) != hipSuccess || hipMalloc(&b, (size_t)blocks * 1024 * 16) != hipSuccess)
        return 1;
    (void)hipMemset(a, 0, (size_t)blocks * 1024 * 16);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int k = 0; k < 3; ++k) {
        for (int w = 0; w < 200; ++w) hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(128), 0, 0, a, b);
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < reps; ++r) {
            if (k == 0) hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(128), 0, 0, (float*)b);
            if (k == 1) hipLaunchKernelGGL(k_load, dim3(blocks), dim3(128), 0, 0, a, (float*)b);
            if (k == 2) hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(128), 0, 0, a, b);
        }
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        std::printf("%s: %.2f us per launch\n", k == 0 ? "empty" : (k == 1 ? "load 16 KiB/WG" : "load+store 16 KiB/WG"),
                    1e3f * ms / reps);
    }
    (void)hipFree(a);
    (void)hipFree(b);
    return 0;
}
