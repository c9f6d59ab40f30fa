// Internal declarations shared by the C-ABI layer (ocean_abi.cpp) and the HIP
// kernel translation units (spectrum.hip, fft2/3/4k.hip, mips.hip).  Not part of the ABI.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ocean/ocean.h"

namespace ocean {

// Kernel timing (ocean_set_kernel_timing): the C-ABI layer points this thread's slot at an
// event pair around one entry point's launches; every kernel launch goes through launch(),
// which attaches the pair to the dispatch itself (hipExtLaunchKernel: start of the first
// kernel, end of the last), so the measured time is the kernels' own, as rocprofv3 reports it,
// with no marker packets between them.
struct LaunchEvents {
    hipEvent_t start, stop;
    bool launched;
};
LaunchEvents*& launch_events();  // thread-local slot, ocean_abi.cpp
// Host pointer of the kernel this thread launched last (ocean_kernel_name reports its symbol).
const void*& last_kernel();  // thread-local slot, ocean_abi.cpp

template <class F, class... Args>
inline void launch(F kernel, dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, Args... args) {
    last_kernel() = (const void*)kernel;
    LaunchEvents* e = launch_events();
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, e && !e->launched ? e->start : nullptr,
                          e ? e->stop : nullptr, 0, args...);
    if (e) e->launched = true;
}

constexpr int kMaxCascades = 5;  // the consumer shader caps cascades at 5 (Water.shader:139)


// Device-side view of one context: every texture of every (tile, cascade) unit.
// unit u = tile * C + cascade; each texture is [u][y][x] (see include/ocean/ocean.h).
struct DevView {
    int n;       // grid side N
    int logn;    // log2 N
    int C;       // cascades
    int T;       // tiles
    int units;   // T * C
    int planes;  // 4 (full) or 2 (displacement only)
    bool normals;
    const float2* noise;  // [T][N][N]
    float4* h0;           // [U][N][N]
    float2* h0k;          // [U][N][N] h0(k) alone (= h0.xy); the mirror-pair row pass reads h0(k) and h0(-k) here
    float4* waves;        // [U][N][N]
    float2* plane[4];     // [U][N][N] each; one allocation, plane[p] = plane[0] + p * plane_stride
    size_t plane_stride;  // elements between consecutive planes (U * N * N)
    float4* disp;         // [U][N][N]
    float4* deriv;        // [U][N][N] (full only)
    float4* turb;         // [U][N][N] (full only)
    float4* normal;       // [U][N][N] (normals only)
    const float2* tw;     // [N + 128]: exp(+2 pi i m / N), m < N; then T1[64] = exp(2 pi i lo / N),
                          // T2[64] = exp(2 pi i 64 hi / N) (two-level table for N > 1024)
    const float* casc;    // [C][5] wavelength, cutoff_low, cutoff_high, swell, fade (device)
    float gravity;        // for the per-frame wave-data recompute (fused row pass)
    int tile_w;           // width W of the tile-major layouts below: inter_w(N), or 4 for small jobs
    float2* tplane;       // fused intermediate, P planes x [K][N/W][N][W] (tile-major), stride inter_stride;
                          // K = the units of one chunk of a frame (ocean_abi.cpp chunk_units): every chunk
                          // reuses the same region, so its lines are rewritten in the Infinity Cache
                          // instead of being written back to HBM once per unit
    size_t inter_stride;  // elements between consecutive planes of tplane (K * N * N)
    float* foam;          // foam state, [U][N/W][N][W] (tile-major); TURB is its broadcast RGBA image
    float2* qside;        // three-plane frame (fftq.hip): per unit of a chunk, d0 [N] then srow [N]
    float4* deriv_mips;   // OCEAN_F_MIPS: per slice, levels 1..log2 N concatenated (mip_chain texels)
    float4* turb_mips;
    size_t mip_chain;     // texels per slice chain: sum over L >= 1 of (N >> L)^2
    // column band (ocean_set_column_band): the fused passes store / transform / fill
    // columns x0 <= x < x0 + nx only (rows are still transformed whole); x0 and nx are
    // multiples of the tile widths, full band = (0, N)
    int x0, nx;
    int c0;  // cascade of unit 0 of this view (a sub-view of a unit chunk may start mid-tile)
    // column parity (ocean_set_column_parity): the context computes the columns x = xstr * m + xpar and
    // stores column x at texture / intermediate column m < N / xstr; xstr = 1, xpar = 0 when off
    int xstr, xpar;
    // pass BQ writes DISP with default-policy stores instead of nontemporal ones: the slice stays in the
    // Infinity Cache and is written back while the next pass A runs, when HBM has headroom.  Set by the host
    // where the frame's re-read set plus DISP fits the cache (ocean_abi.cpp disp_fits_cache).
    bool disp_cached;
};

struct SpectrumParams {
    float wind_speed, wind_dir_x, wind_dir_y, gravity, fetch, depth;
};

// spectrum.hip
// Resident workgroups per CU of `kernel` at `threads` lanes (hipOccupancyMaxActiveBlocksPerMultiprocessor,
// at least 1) and the device's CU count, cached per device (and kernel): the queries cost microseconds
// of host time, paid once instead of per launch (small jobs issue a launch every few microseconds).
int resident_per_cu(const void* kernel, int threads);
int device_cus();

hipError_t launch_init_spectrum(const DevView& v, const SpectrumParams& p, hipStream_t s);
hipError_t launch_conjugate(const DevView& v, hipStream_t s);
hipError_t launch_evolve(const DevView& v, float t, hipStream_t s);
hipError_t launch_fill(const DevView& v, hipStream_t s);
hipError_t launch_foam_import(const DevView& v, hipStream_t s);
hipError_t launch_noise(const DevView& v, uint64_t seed, hipStream_t s);
// h0k = h0.xy (a context whose h0k is allocated after its spectrum: ocean_set_column_parity)
hipError_t launch_h0k_extract(const DevView& v, hipStream_t s);

// fft2.hip: the operator IFFT (IFFT.InverseFastFourierTransform): persistent,
// software-pipelined row and column(+permute) launches, in place.
// Entries of the per-stage twiddle tables stored at tw + N + 128 (see fft_engine.h StageTw).
size_t stage_twiddle_entries(int n);
// Each launch covers `ups` consecutive unit-planes from `base` (plane p of unit u is unit-plane
// p * U + u of the one plane allocation), in place.
hipError_t launch_ifft_rows_v2(const DevView& v, float2* base, int ups, hipStream_t s);
hipError_t launch_ifft_cols_v2(const DevView& v, float2* base, int ups, hipStream_t s);
// N = 4096: the operator over `ups` consecutive unit-planes at `planes` (plane p of unit u is
// unit-plane p * U + u) with its column transform split by decimation in frequency into two 2048-point
// column transforms, in place (fft2.hip): part 0 = rows + fold onto the planes' own rows (k_rowsf),
// 1 = the column transforms + permute, both sub-planes of an XCD-paired 8-column tile per item (k_colsf_ip).
hipError_t launch_ifft_fold(const DevView& v, float2* planes, int ups, int part, hipStream_t s);

// fft3.hip: fused frame through the tile-major intermediate; the row pass
// recomputes wave data and feeds evolve straight into a radix-4/8 first stage;
// the column pass (N <= 1024) reads contiguous tiles and the compact foam state.
hipError_t launch_pass_a_v3(const DevView& v, float t, hipStream_t s);
hipError_t launch_pass_b_v3(const DevView& v, hipStream_t s);
// mips.hip: box-filter mip chains of DERIV and TURB (OCEAN_F_MIPS)
hipError_t launch_mips(const DevView& v, hipStream_t s);
// mips.hip: DISP.y of one slice compacted to float[N][N] (ocean_read_height_async); texels % 4 == 0
hipError_t launch_extract_height(const float4* disp_slice, float* dst, size_t texels, hipStream_t s);
// sample.hip: cascade-summed world sampling (Water.shader:314-348), device pointers
hipError_t launch_sample_world(const DevView& v, int tile, const float* pts, int count, float* out, hipStream_t s);

// fft4k.hip (N = 2048, 4096): four-step column passes C1 (in place on the
// 16-wide tile-major intermediate) + C2 (with the pass-B epilogue); replace pass B.
bool pass_c4_supported(int n);
hipError_t launch_pass_c4(const DevView& v, hipStream_t s);
// Mirror-pair row pass (N = 512 / 1024, 4 planes): one item = rows y and N - y; the
// texels k and -k share wave data and the phase factor and read h0 once (h0k).
bool pass_a4_supported(int n, int planes);
hipError_t launch_pass_a_v4(const DevView& v, float t, hipStream_t s);
// fftq.hip: the fused frame through a three-plane intermediate (full outputs): pass AQ
// (mirror-pair rows, N = 512 / 1024) or A3Q (one row per item, N = 2048 / 4096), then pass BQ
// (column tiles, four transforms, N <= 1024) or the four-step column passes with Q planes.
bool pass_q_supported(int n, int planes);
hipError_t launch_pass_a_q(const DevView& v, float t, hipStream_t s);
hipError_t launch_pass_b_q(const DevView& v, hipStream_t s);
// fft4k.hip with the three-plane intermediate: C1 also forms and transforms R[Q4] into the fourth
// plane slot; C2 runs the three-plane epilogue.
hipError_t launch_pass_c4q(const DevView& v, hipStream_t s);

}  // namespace ocean
