// HBM ceilings of the operator IFFT's access shapes beyond the 256 MiB Infinity Cache.
// Build: hipcc --offload-arch=gfx950 -O3 tools/hbmbench.hip -o tools/hbmbench
// Every test streams a buffer of `MiB` (default 512) once per launch; prints the
// bytes read + written per launch / average launch time (HIP events, 20 launches).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

// in place: x = x * s over float4 (grid-stride)
__global__ void k_inplace4(float4* __restrict__ a, size_t n, float s) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        a[i] = make_float4(v.x * s, v.y * s, v.z * s, v.w * s);
    }
}
// out of place copy float4
__global__ void k_copy4(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
// read only (sum) float4
__global__ void k_read4(const float4* __restrict__ a, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;
}
// write only float4
__global__ void k_write4(float4* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}
// in place, rows of 1024 float2 (8 KiB), 4 rows per 256-lane workgroup, 16 values per lane
// held in registers before any store (the row pass's shape without the FFT)
__global__ void k_rows_shape(float2* __restrict__ a, size_t rows) {
    for (size_t r0 = (size_t)blockIdx.x * 4; r0 < rows; r0 += (size_t)gridDim.x * 4) {
        float2* p = a + r0 * 1024;
        float2 v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = p[threadIdx.x + i * 256];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) p[threadIdx.x + i * 256] = make_float2(v[i].x * 0.5f, v[i].y);
    }
}

template <class F>
float time_it(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? std::atoi(argv[1]) : 512;
    const size_t bytes = mib << 20;
    const size_t n4 = bytes / 16;
    float4 *a = nullptr, *b = nullptr;
    float* o = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&o, 4));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int per_cu : {4, 8, 16}) {
        const int g = cus * per_cu;
        float us = time_it([&] { k_inplace4<<<g, 256>>>(a, n4, 1.0f); }, 20);
        printf("inplace4 %zu MiB grid %d  %.1f us  %.1f GB/s\n", mib, g, us, 2.0 * bytes / us / 1e3);
        us = time_it([&] { k_copy4<<<g, 256>>>(a, b, n4); }, 20);
        printf("copy4    %zu MiB grid %d  %.1f us  %.1f GB/s\n", mib, g, us, 2.0 * bytes / us / 1e3);
        us = time_it([&] { k_read4<<<g, 256>>>(a, n4, o); }, 20);
        printf("read4    %zu MiB grid %d  %.1f us  %.1f GB/s\n", mib, g, us, 1.0 * bytes / us / 1e3);
        us = time_it([&] { k_write4<<<g, 256>>>(a, n4); }, 20);
        printf("write4   %zu MiB grid %d  %.1f us  %.1f GB/s\n", mib, g, us, 1.0 * bytes / us / 1e3);
        us = time_it([&] { k_rows_shape<<<g, 256>>>((float2*)a, bytes / 8192); }, 20);
        printf("rows     %zu MiB grid %d  %.1f us  %.1f GB/s\n", mib, g, us, 2.0 * bytes / us / 1e3);
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    return 0;
}
