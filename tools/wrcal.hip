// Calibration of rocprofv3's WRITE_SIZE for the 4096 operator column launch's store shape (VERDICT r05 item 5:
// k_colsf_ip's WRITE_SIZE is 1.16x its algorithmic bytes).  MI355X_MICROARCH.md: WRITE_SIZE reads the
// bytes exactly only for 16-B-per-lane streaming stores; k_colsf_ip stores 8 B per lane in 64-B row
// pieces (8-column tiles, XCD-paired halves of 128-B lines).  Each kernel writes the same 256 MiB of a
// 4096-wide float2 plane set; the program prints each one's time (HIP events), rocprofv3 --pmc gives
// WRITE_SIZE / TCC_EA0_WRREQ per kernel.
//   0  16 B per lane, contiguous                 (the calibrated shape)
//   1  8 B per lane, contiguous                  (whole lines, 8-B lanes)
//   2  8-column tiles, halves paired on one XCD  (k_colsf_ip's shape), default policy
//   3  the same, nontemporal                     (k_colsf_ip's three directly stored quarters)
//   4  16-column tiles, one workgroup per line   (whole lines in one instruction), default policy
//   5  the same, nontemporal
// Build: hipcc --offload-arch=gfx950 -O3 tools/wrcal.hip -o tools/wrcal
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
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int N = 4096;            // plane width (texels)
constexpr size_t kBytes = 256u << 20;
constexpr size_t kRows = kBytes / (N * 8);  // 8192 rows of 4096 float2

__global__ void k_contig16(f32x4* out, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        out[i] = f32x4{1.0f, 2.0f, 3.0f, (float)i};
}
__global__ void k_contig8(f32x2* out, size_t n2) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x)
        out[i] = f32x2{1.0f, (float)i};
}
// W-column tiles of 1024 lanes: lane (b = tid % W, j = tid / W); a tile covers W columns x (1024 / W) rows
// per step and walks down its columns.  W = 8: tiles t and its partner t ^ 1 (the other half of each
// 128-B line) run as blocks b and b + 8 (one XCD under round-robin placement), as k_colsf_ip's G = 2.
template <int W, bool NT>
__global__ __launch_bounds__(1024) void k_tiles(f32x2* out, int tiles_total) {
    const int lb = threadIdx.x % W, lj = threadIdx.x / W;
    constexpr int RPS = 1024 / W;  // rows per step
    for (int item = blockIdx.x; item < tiles_total; item += gridDim.x) {
        int t = item;
        if (W == 8) t = (item & ~15) + 2 * (item & 7) + ((item >> 3) & 1);  // blocks b, b + 8 -> tiles 2k, 2k + 1
        const int col_tiles = N / W;
        const int tile_col = t % col_tiles, band = t / col_tiles;  // band: a group of rows
        const size_t row0 = (size_t)band * 2048;
        for (int s = 0; s < 2048 / RPS; ++s) {
            const size_t row = row0 + (size_t)s * RPS + lj;
            f32x2* p = out + row * N + (size_t)tile_col * W + lb;
            const f32x2 v = {(float)row, (float)lb};
            if constexpr (NT) __builtin_nontemporal_store(v, p);
            else *p = v;
        }
    }
}

template <class F>
int timed(const char* name, int id, F&& launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();  // warm
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"kernel\": %d, \"shape\": \"%s\", \"us\": %.2f, \"TBs\": %.3f}\n", id, name, ms * 1e3f / 5,
           kBytes / (ms * 1e-3 / 5) / 1e12);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return 0;
}

int main() {
    f32x2* out;
    CK(hipMalloc(&out, kBytes));
    const int tiles8 = (int)((N / 8) * (kRows / 2048)), tiles16 = (int)((N / 16) * (kRows / 2048));
    const int g = 256;  // one 1024-lane workgroup per CU, as k_colsf_ip
    if (timed("contig16", 0, [&] { hipLaunchKernelGGL(k_contig16, dim3(4096), dim3(256), 0, 0, (f32x4*)out, kBytes / 16); }) ||
        timed("contig8", 1, [&] { hipLaunchKernelGGL(k_contig8, dim3(4096), dim3(256), 0, 0, out, kBytes / 8); }) ||
        timed("tiles8", 2, [&] { hipLaunchKernelGGL((k_tiles<8, false>), dim3(g), dim3(1024), 0, 0, out, tiles8); }) ||
        timed("tiles8_nt", 3, [&] { hipLaunchKernelGGL((k_tiles<8, true>), dim3(g), dim3(1024), 0, 0, out, tiles8); }) ||
        timed("tiles16", 4, [&] { hipLaunchKernelGGL((k_tiles<16, false>), dim3(g), dim3(1024), 0, 0, out, tiles16); }) ||
        timed("tiles16_nt", 5, [&] { hipLaunchKernelGGL((k_tiles<16, true>), dim3(g), dim3(1024), 0, 0, out, tiles16); }))
        return 1;
    CK(hipFree(out));
    return 0;
}
