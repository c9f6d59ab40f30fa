// Probe: does hipExtAnyOrderLaunch let a kernel's workgroups start before the previous kernel on the
// same stream has finished (AQL barrier bit clear)?  hip_ext.h says the flag is "not supported on AMD
// GFX9xx boards" for hipExtModuleLaunchKernel; this measures what hipExtLaunchKernel does on gfx950.
// K1: 512 workgroups, workgroup b busy-waits (wall clock) 5 + b * 0.05 us, then records its end time.
// K2: 256 workgroups record their start time.  Printed: K2's first start minus K1's last end (negative =
// overlap), for a plain launch of K2 and for an any-order launch, 5 repetitions each.
// Every wait is bounded by the wall clock (<= 40 us), so nothing can hang.
// Build: hipcc --offload-arch=gfx950 -O3 tools/anyorder_probe.hip -o tools/anyorder_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

// wall_clock64() ticks at 100 MHz on MI300-class parts (10 ns)
__global__ void k_busy(unsigned long long* end_t, int base_ticks, int step_ticks) {
    const unsigned long long t0 = wall_clock64();
    const unsigned long long until = t0 + (unsigned long long)(base_ticks + step_ticks * (int)blockIdx.x);
    while (wall_clock64() < until) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0) end_t[blockIdx.x] = wall_clock64();
}

__global__ void k_mark(unsigned long long* start_t) {
    if (threadIdx.x == 0) start_t[blockIdx.x] = wall_clock64();
}

int main() {
    constexpr int G1 = 512, G2 = 256;
    unsigned long long *e1, *s2;
    CK(hipMalloc(&e1, G1 * 8));
    CK(hipMalloc(&s2, G2 * 8));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    std::vector<unsigned long long> he(G1), hs(G2);
    for (int rep = 0; rep < 5; ++rep) {
        for (int flag = 0; flag < 2; ++flag) {
            hipLaunchKernelGGL(k_busy, dim3(G1), dim3(256), 0, st, e1, 500, 5);  // 5 us + b * 0.05 us
            CK(hipGetLastError());
            void* args[] = {&s2};
            CK(hipExtLaunchKernel((const void*)k_mark, dim3(G2), dim3(256), args, 0, st, nullptr, nullptr,
                                  flag ? hipExtAnyOrderLaunch : 0));
            CK(hipStreamSynchronize(st));
            CK(hipMemcpy(he.data(), e1, G1 * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hs.data(), s2, G2 * 8, hipMemcpyDeviceToHost));
            const unsigned long long last_end = *std::max_element(he.begin(), he.end());
            const unsigned long long first_end = *std::min_element(he.begin(), he.end());
            const unsigned long long first_start = *std::min_element(hs.begin(), hs.end());
            printf("{\"rep\": %d, \"any_order\": %d, \"k2_first_start_minus_k1_last_end_us\": %.2f, "
                   "\"k1_end_spread_us\": %.2f}\n",
                   rep, flag, ((double)first_start - (double)last_end) * 0.01, ((double)last_end - (double)first_end) * 0.01);
        }
    }
    CK(hipFree(e1));
    CK(hipFree(s2));
    CK(hipStreamDestroy(st));
    return 0;
}
