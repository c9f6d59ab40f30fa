// Mip chains of DERIV and TURB (OCEAN_F_MIPS): GenerateMips of WaterBody.cs:191-192
// on the two mip-mapped texture arrays (WaterBody.cs:228-229).  Box filter,
// texel = ((a + b) + (c + d)) * 0.25 of the 2x2 texels below (ocean.h).
//
// k_mips_block: one workgroup per 32x32 block of level 0 of one slice builds
//   levels 1..5 of that block through LDS (each level 0 texel read once; TURB's from the foam state).
// k_mips_tail: one workgroup per slice builds the remaining levels from level 5.
// Bytes per texel-cascade: read DERIV (16 B) and the foam state (4 B), write 1/3 of 32 B.
#include <algorithm>

#include "ocean_internal.h"

namespace ocean {
namespace {

constexpr int kBlk = 32;  // level-0 block per workgroup (levels 1..5)

__device__ __forceinline__ float4 box(float4 a, float4 b, float4 c, float4 d) {
    return make_float4(((a.x + b.x) + (c.x + d.x)) * 0.25f, ((a.y + b.y) + (c.y + d.y)) * 0.25f,
                       ((a.z + b.z) + (c.z + d.z)) * 0.25f, ((a.w + b.w) + (c.w + d.w)) * 0.25f);
}

// DERIV's level 0 is read with nontemporal loads: it is read once here, and default-policy loads of its 64 MiB
// (cfg3) evicted pass A's h0k from the Infinity Cache (pass A 30-35 -> 29 us in the Update loop;
// docs/MEASUREMENTS.md section 9).
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_nt(const float4* p) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ size_t mip_off(int n, int level) {  // texels before `level` in a chain
    size_t o = 0;
    for (int l = 1; l < level; ++l) o += (size_t)(n >> l) * (n >> l);
    return o;
}

// grid: (blocks per slice, slices, 2 textures); 256 lanes, lane t -> texel (t % h, t / h) of the h x h
// level-1 block, h = blk / 2.
__global__ __launch_bounds__(256) void k_mips_block(DevView v, int blk, int levels) {
    const int n = v.n;
    const int tex = blockIdx.z;
    const float4* src = v.deriv + (size_t)blockIdx.y * n * n;
    float4* chain = (tex == 0 ? v.deriv_mips : v.turb_mips) + (size_t)blockIdx.y * v.mip_chain;
    const int bpr = n / blk;  // blocks per row
    const int bx = blockIdx.x % bpr, by = blockIdx.x / bpr;
    __shared__ float4 cur[kBlk / 2 * kBlk / 2];
    int h = blk / 2;
    const int m1 = n >> 1;
    for (int t = threadIdx.x; t < h * h; t += blockDim.x) {
        const int x = t % h, y = t / h;
        const int X = bx * blk + 2 * x, Y = by * blk + 2 * y;
        float4 r;
        if (tex == 1) {
            // TURB is the broadcast RGBA image of the foam state (ResultTexturesFiller.compute:32; every fill and
            // ocean_write of TURB keeps the two equal), so its level 1 is boxed from the 4-byte state: the same
            // sums of the same values as boxing TURB's four equal channels, a quarter of the bytes.  State layout
            // [u][x/W][y][W]: texels X, X + 1 are adjacent in a tile row (X even, W even), row Y + 1 is W on.
            const int W = v.tile_w;
            const float* fs = v.foam + (size_t)blockIdx.y * n * n + ((size_t)(X / W) * n + Y) * W + (X % W);
            const float2 ab = *reinterpret_cast<const float2*>(fs), cd = *reinterpret_cast<const float2*>(fs + W);
            const float f = ((ab.x + ab.y) + (cd.x + cd.y)) * 0.25f;
            r = make_float4(f, f, f, f);
        } else {
            const float4* p = src + (size_t)Y * n + X;
            r = box(ld_nt(p), ld_nt(p + 1), ld_nt(p + n), ld_nt(p + n + 1));
        }
        chain[mip_off(n, 1) + (size_t)(by * h + y) * m1 + bx * h + x] = r;
        cur[t] = r;
    }
    for (int level = 2; level <= levels; ++level) {
        __syncthreads();
        const int hp = h;
        h >>= 1;
        float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
        const bool act = (int)threadIdx.x < h * h;
        if (act) {
            const int x = threadIdx.x % h, y = threadIdx.x / h;
            r = box(cur[(2 * y) * hp + 2 * x], cur[(2 * y) * hp + 2 * x + 1], cur[(2 * y + 1) * hp + 2 * x],
                    cur[(2 * y + 1) * hp + 2 * x + 1]);
            chain[mip_off(n, level) + (size_t)(by * h + y) * (n >> level) + bx * h + x] = r;
        }
        __syncthreads();
        if (act) cur[threadIdx.x] = r;
    }
}

// grid: (slices, 2 textures); levels first..log2 n from level first-1 in the chain.  Levels whose source is
// larger than kBlk x kBlk (N > 1024) are built from the chain in global memory; from the first source that
// fits, it is read once into LDS and every further level is built there (one global read round trip instead
// of one per level: 6.28 -> 5.76 us per cfg3 frame, docs/MEASUREMENTS.md section 9).
__global__ __launch_bounds__(256) void k_mips_tail(DevView v, int first) {
    const int n = v.n;
    const int tex = blockIdx.y;
    float4* chain = (tex == 0 ? v.deriv_mips : v.turb_mips) + (size_t)blockIdx.x * v.mip_chain;
    __shared__ float4 lv[2][kBlk * kBlk];  // ping-pong images of consecutive levels
    int level = first;
    for (; (n >> (level - 1)) > kBlk; ++level) {  // source too large for the LDS image
        const int m = n >> level, mp = n >> (level - 1);
        const float4* s = chain + mip_off(n, level - 1);
        float4* d = chain + mip_off(n, level);
        for (int t = threadIdx.x; t < m * m; t += blockDim.x) {
            const int x = t % m, y = t / m;
            d[t] = box(s[(2 * y) * mp + 2 * x], s[(2 * y) * mp + 2 * x + 1], s[(2 * y + 1) * mp + 2 * x],
                       s[(2 * y + 1) * mp + 2 * x + 1]);
        }
        __syncthreads();
    }
    int mp = n >> (level - 1);
    const float4* s0 = chain + mip_off(n, level - 1);
    for (int t = threadIdx.x; t < mp * mp; t += blockDim.x) lv[0][t] = s0[t];
    int cur = 0;
    for (; (n >> level) >= 1; ++level) {
        __syncthreads();
        const int m = n >> level;
        const float4* src = lv[cur];
        float4* dst = lv[cur ^ 1];
        float4* d = chain + mip_off(n, level);
        for (int t = threadIdx.x; t < m * m; t += blockDim.x) {
            const int x = t % m, y = t / m;
            const float4 r = box(src[(2 * y) * mp + 2 * x], src[(2 * y) * mp + 2 * x + 1], src[(2 * y + 1) * mp + 2 * x],
                                 src[(2 * y + 1) * mp + 2 * x + 1]);
            dst[t] = r;
            d[t] = r;
        }
        cur ^= 1;
        mp = m;
    }
}

// The height channel (.y = Dy, what GetWaterHeight reads: WaterBody.cs:208) of one DISP slice, compacted
// to float[N][N] for ocean_read_height_async: a quarter of the RGBA slice's bytes over the link.  Four
// texels per lane: 64 B read, 16 B written.
__global__ __launch_bounds__(256) void k_extract_height(const float4* __restrict__ src, float4* __restrict__ dst,
                                                        size_t quads) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < quads; i += (size_t)gridDim.x * blockDim.x) {
        const float4 a = src[4 * i], b = src[4 * i + 1], c = src[4 * i + 2], d = src[4 * i + 3];
        dst[i] = make_float4(a.y, b.y, c.y, d.y);
    }
}

}  // namespace

hipError_t launch_extract_height(const float4* disp_slice, float* dst, size_t texels, hipStream_t s) {
    if (texels % 4 != 0) return hipErrorInvalidValue;
    const size_t quads = texels / 4;
    const int g = (int)std::min<size_t>((quads + 255) / 256, 4096);
    launch(k_extract_height, dim3(g), dim3(256), 0, s, disp_slice, reinterpret_cast<float4*>(dst), quads);
    return hipGetLastError();
}

hipError_t launch_mips(const DevView& v, hipStream_t s) {
    if (!v.deriv_mips || !v.turb_mips || !v.foam) return hipErrorInvalidValue;
    const int n = v.n;
    const int blk = n < kBlk ? n : kBlk;
    int levels = 0;
    while ((1 << levels) < blk) ++levels;  // levels 1..log2(blk) from the block kernel
    if (v.tile_w < 2 || v.tile_w % 2) return hipErrorInvalidValue;  // foam-state texel pairs (k_mips_block)
    const int bps = (n / blk) * (n / blk);
    launch(k_mips_block, dim3(bps, v.units, 2), dim3(256), 0, s, v, blk, levels);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    if (blk < n) {
        launch(k_mips_tail, dim3(v.units, 2), dim3(256), 0, s, v, levels + 1);
        return hipGetLastError();
    }
    return hipSuccess;
}

}  // namespace ocean
