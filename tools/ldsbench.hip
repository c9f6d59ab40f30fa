// LDS access patterns of pass AQ (fftq.hip) and the 4096 operator's row launch (fft4k.hip), one kernel
// per pattern, to read SQ_LDS_BANK_CONFLICT per pattern: the same instruction forms
// the kernels compile to (ds_read2_b64 / ds_write2_b64 / ds_read2st64_b64, checked in the asm), on
// the kernels' padded image (one complex per 16: pad(i) = i + i / 16), 256 lanes = four waves, one
// workgroup per CU.  Run under rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS;
// the program prints each kernel's time.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ldsbench.hip -o tools/ldsbench
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

constexpr int kImage = 4 * 1088 + 256;  // four padded 1024-point sequences
__host__ __device__ constexpr int pad(int i) { return i + i / 16; }
__host__ __device__ constexpr int loff(int k, int rs) { return k * rs + (k * rs) / 16; }
// swizzled alternative: one complex every 32 (i + i / 32)
__host__ __device__ constexpr int pad32(int i) { return i + i / 32; }

// PAT  what                                                       pass AQ / rowsf source
//  0   stage read: elements b*1024 + j + 64 r, r < 16 (ds_read2_b64)  stages_from, RD = 64
//  1   the same, four reads 256 apart (single ds_read_b64 each)
//  2   stage write: elements y0 + 4 q, y0 = (j/4)*64 + j%4           stages_from ST = 1, WR = 4
//  3   put: elements 4 j + q, q < 4                                  put(b, j)
//  4   put mirrored: 4 jm + q, jm = (256 - j) % 256                  put(b, jm)
//  5   stage-2 twiddles: entry j + 64 r (ds_read2st64_b64)            StageTw::apply<2>
//  6   contiguous ds_read_b64 (element j): the conflict-free floor
//  7   stage read on pad32                                           candidate
//  8   stage write on pad32                                          candidate
//  9   put on pad32                                                  candidate
template <int PAT>
__global__ __launch_bounds__(256) void k_lds(float2* out, int iters) {
    __shared__ float2 lds[kImage];
    const int t = (int)threadIdx.x, j = t & 63, b = t >> 6, jl = t;  // jl: lane of a 256-lane put
    for (int i = t; i < kImage; i += 256) lds[i] = make_float2((float)i, (float)-i);
    __syncthreads();
    float ax = 0.0f, ay = 0.0f;
    for (int it = 0; it < iters; ++it) {
        if constexpr (PAT == 0 || PAT == 7) {
            const float2* src = lds + (PAT == 0 ? pad(b * 1024 + j) : 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float2 x = PAT == 0 ? src[loff(r, 64)] : lds[pad32(b * 1024 + j + 64 * r)];
                ax += x.x;
                ay += x.y;
            }
        } else if constexpr (PAT == 1) {
            const float2* src = lds + pad(b * 1024 + j);
#pragma unroll
            for (int r = 0; r < 16; r += 4) {
                const float2 x = src[loff(r, 64)];
                ax += x.x;
                ay += x.y;
            }
        } else if constexpr (PAT == 2 || PAT == 8) {
            const int y0 = (j / 4) * 64 + (j & 3);
            float2* dst = lds + pad(b * 1024 + y0);
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                if constexpr (PAT == 2) dst[loff(q, 4)] = make_float2(ax + q, ay);
                else lds[pad32(b * 1024 + y0 + 4 * q)] = make_float2(ax + q, ay);
            }
        } else if constexpr (PAT == 3 || PAT == 4 || PAT == 9) {
            const int jj = PAT == 4 ? ((256 - jl) & 255) : jl;
            // four sequences' puts, as put(k, .) for k < 4 (the lanes cover butterflies 0..255)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float2* dst = lds + (PAT == 9 ? pad32(k * 1024 + jj * 4) : pad(k * 1024 + jj * 4));
#pragma unroll
                for (int q = 0; q < 4; ++q) dst[q] = make_float2(ax + q, ay + k);
            }
        } else if constexpr (PAT == 5) {
            const float2* tw = lds + 100 + j;
#pragma unroll
            for (int r = 1; r < 16; ++r) {
                const float2 x = tw[r * 64];
                ax += x.x;
                ay += x.y;
            }
        } else if constexpr (PAT == 6) {
            const float2* src = lds + pad(b * 1024) + j;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float2 x = src[r * 68];
                ax += x.x;
                ay += x.y;
            }
        }
        __asm__ volatile("" ::: "memory");
    }
    __syncthreads();
    out[blockIdx.x * 256 + t] = make_float2(ax + lds[t].x, ay);
}

template <int PAT>
int run(float2* out, int blocks, int iters) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_lds<PAT>, dim3(blocks), dim3(256), 0, 0, out, iters);  // warm
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_lds<PAT>, dim3(blocks), dim3(256), 0, 0, out, iters);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"pattern\": %d, \"us\": %.2f, \"blocks\": %d, \"iters\": %d}\n", PAT, ms * 1e3f, blocks, iters);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return 0;
}

int main() {
    const int blocks = 256, iters = 256;
    float2* out;
    CK(hipMalloc(&out, blocks * 256 * sizeof(float2)));
    if (run<0>(out, blocks, iters) || run<1>(out, blocks, iters) || run<2>(out, blocks, iters) ||
        run<3>(out, blocks, iters) || run<4>(out, blocks, iters) || run<5>(out, blocks, iters) ||
        run<6>(out, blocks, iters) || run<7>(out, blocks, iters) || run<8>(out, blocks, iters) ||
        run<9>(out, blocks, iters))
        return 1;
    CK(hipFree(out));
    return 0;
}
