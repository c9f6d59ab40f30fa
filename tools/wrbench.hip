// Write-side ceilings of pass B's traffic on MI355X (docs/MEASUREMENTS.md section 3, "where the frame's time
// goes"): (1) streamed float4 stores alone, nontemporal and default policy, over pass B's 192 MiB
// of textures; (2) a re-read of a 96 MiB buffer (the three-plane intermediate, Infinity-Cache
// resident after its first pass) alone; (3) both at once in one kernel, the byte mix of pass BQ.
// Build: hipcc --offload-arch=gfx950 -O3 tools/wrbench.hip -o tools/wrbench
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

template <bool NT>
__global__ void k_write(f32x4* __restrict__ out, size_t n4, float s) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const f32x4 v = {s, s + 1.0f, s + 2.0f, (float)i};
        if constexpr (NT) __builtin_nontemporal_store(v, out + i);
        else out[i] = v;
    }
}

// write-through (sc1) float4 stores
__global__ void k_write_sc1(f32x4* __restrict__ out, size_t n4, float s) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const f32x4 v = {s, s + 1.0f, s + 2.0f, (float)i};
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(out + i), "v"(v) : "memory");
    }
}

__global__ void k_read(const f32x4* __restrict__ in, size_t n4, float* sink) {
    f32x4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        acc += in[i];
    if (acc.x == 12345.0f) sink[0] = acc.y;  // keeps the loads
}

// pass BQ's mix: per 16-B read of the intermediate, 32 B of nontemporal texture stores.  k_mix
// interleaves the two stores of a lane (32-B lane stride: every store instruction writes half of
// each line it touches); k_mix2 writes two contiguous streams (whole lines, as pass BQ's textures).
__global__ void k_mix(const f32x4* __restrict__ in, f32x4* __restrict__ out, size_t n4in) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4in; i += (size_t)gridDim.x * blockDim.x) {
        const f32x4 v = in[i];
        __builtin_nontemporal_store(v, out + 2 * i);
        __builtin_nontemporal_store(v * 2.0f, out + 2 * i + 1);
    }
}
__global__ void k_mix2(const f32x4* __restrict__ in, f32x4* __restrict__ out, size_t n4in) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4in; i += (size_t)gridDim.x * blockDim.x) {
        const f32x4 v = in[i];
        __builtin_nontemporal_store(v, out + i);
        __builtin_nontemporal_store(v * 2.0f, out + n4in + i);
    }
}

int main() {
    const size_t out_bytes = (size_t)192 << 20, in_bytes = (size_t)96 << 20;
    f32x4 *out, *in;
    float* sink;
    CK(hipMalloc(&out, out_bytes));
    CK(hipMalloc(&in, in_bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(in, 0, in_bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int reps = 50;
    {  // beyond the Infinity Cache: 1 GiB written per launch, plain / nontemporal / write-through
        const size_t big = (size_t)1 << 30;
        f32x4* o2;
        CK(hipMalloc(&o2, big));
        for (int mode = 0; mode < 3; ++mode) {
            auto run = [&]() {
                if (mode == 0) hipLaunchKernelGGL(k_write<false>, dim3(4096), dim3(256), 0, 0, o2, big / 16, 1.0f);
                if (mode == 1) hipLaunchKernelGGL(k_write<true>, dim3(4096), dim3(256), 0, 0, o2, big / 16, 1.0f);
                if (mode == 2) hipLaunchKernelGGL(k_write_sc1, dim3(4096), dim3(256), 0, 0, o2, big / 16, 1.0f);
            };
            for (int w = 0; w < 3; ++w) run();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int r = 0; r < 10; ++r) run();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const char* names[] = {"write plain 1 GiB", "write nt 1 GiB", "write sc1 1 GiB"};
            printf("%-24s grid  4096 %8.1f us %8.1f GB/s\n", names[mode], ms * 1e2, (double)big / (ms * 1e2) / 1e3);
        }
        CK(hipFree(o2));
    }
    for (int grid : {2048}) {
        for (int mode = 0; mode < 6; ++mode) {
            auto run = [&]() {
                if (mode == 4) hipLaunchKernelGGL(k_write_sc1, dim3(grid), dim3(256), 0, 0, out, out_bytes / 16, 1.0f);
                if (mode == 0) hipLaunchKernelGGL(k_write<true>, dim3(grid), dim3(256), 0, 0, out, out_bytes / 16, 1.0f);
                if (mode == 1) hipLaunchKernelGGL(k_write<false>, dim3(grid), dim3(256), 0, 0, out, out_bytes / 16, 1.0f);
                if (mode == 2) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, in, in_bytes / 16, sink);
                if (mode == 3) hipLaunchKernelGGL(k_mix, dim3(grid), dim3(256), 0, 0, in, out, in_bytes / 16);
                if (mode == 5) hipLaunchKernelGGL(k_mix2, dim3(grid), dim3(256), 0, 0, in, out, in_bytes / 16);
            };
            for (int w = 0; w < 5; ++w) run();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int r = 0; r < reps; ++r) run();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const double us = ms * 1e3 / reps;
            const double bytes = mode == 2 ? in_bytes : ((mode == 3 || mode == 5) ? in_bytes + out_bytes : out_bytes);
            const char* names[] = {"write nt 192 MiB", "write plain 192 MiB", "re-read 96 MiB", "read 96 + write nt 192",
                                   "write sc1 192 MiB", "read 96 + nt 192 lines"};
            printf("%-24s grid %5d %8.1f us %8.1f GB/s\n", names[mode], grid, us, bytes / us / 1e3);
        }
    }
    return 0;
}
