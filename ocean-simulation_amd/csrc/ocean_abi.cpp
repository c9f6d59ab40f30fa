// C-ABI layer of liboceanhip.so: context lifetime, validation, device memory,
// the per-frame schedule, readback and kernel timing.  See include/ocean/ocean.h
// for the reference interface each entry point replaces.
#include <cxxabi.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <string>
#include <vector>

#include "fft_core.h"
#include "device_scope.h"
#include "ocean_internal.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(OCEAN_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

#define OCEAN_HIP(call)                                   \
    do {                                                  \
        hipError_t _e = (call);                           \
        if (_e != hipSuccess) return hip_fail(_e, #call); \
    } while (0)

struct TimedLaunch {
    int kind;
    hipEvent_t a, b;
};

}  // namespace

namespace ocean {
LaunchEvents*& launch_events() {
    thread_local LaunchEvents* slot = nullptr;
    return slot;
}
const void*& last_kernel() {
    thread_local const void* slot = nullptr;
    return slot;
}

namespace {
std::mutex g_occ_mu;
std::map<std::tuple<int, const void*, int>, int> g_occ;  // (device, kernel, threads) -> per CU
std::map<int, int> g_cus;                                 // device -> CUs
int current_device() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    return dev;
}
}  // namespace

int resident_per_cu(const void* kernel, int threads) {
    const auto key = std::make_tuple(current_device(), kernel, threads);
    std::lock_guard<std::mutex> lk(g_occ_mu);
    auto it = g_occ.find(key);
    if (it != g_occ.end()) return it->second;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu <= 0)
        per_cu = 1;
    g_occ.emplace(key, per_cu);
    return per_cu;
}

int device_cus() {
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(g_occ_mu);
    auto it = g_cus.find(dev);
    if (it != g_cus.end()) return it->second;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    g_cus.emplace(dev, cus);
    return cus;
}
}  // namespace ocean

// Host noise generator (WaterBody.cs:71-100 with this library's documented
// uniform source).  Defined in noise.cpp.
namespace ocean {
void generate_noise_host(int n, uint64_t seed, float* out);
}

// Staging slots of ocean_read_async / ocean_read_height_async.  A slot is device memory as large as one
// slice of the largest texture plus the events of the request holding it, created once with the slot: no
// event is created per request.  `after` and `done` disable timing; the timed pair `tstart` / `tdone`
// (ocean_readback_copy_ms) is created on the slot's first request made with readback timing on
// (ocean_set_readback_timing) and recorded only for such requests.  A request takes a slot and gives it back
// when it is released (after its host copy has landed), so a slot is never rewritten while a copy out of
// it is pending, and no allocation or free sits between the context stream and the copy stream.  Shared
// with the requests: it outlives a context destroyed before its requests are released.
struct StageSlot {
    void* mem = nullptr;
    hipEvent_t after = nullptr;  // the snapshot is in the slot (the copy stream waits for it)
    hipEvent_t done = nullptr;   // the host copy has landed (untimed requests)
    hipEvent_t tstart = nullptr, tdone = nullptr;  // timed requests: around the host copy itself
};
struct StagePool {
    int device = 0;
    size_t slot_bytes = 0;
    std::mutex mu;
    std::vector<StageSlot*> free_slots, all;
    ~StagePool() {
        int prev = 0;
        const bool had = hipGetDevice(&prev) == hipSuccess;
        (void)hipSetDevice(device);
        for (StageSlot* sl : all) {
            if (sl->mem) (void)hipFree(sl->mem);
            for (hipEvent_t e : {sl->after, sl->done, sl->tstart, sl->tdone})
                if (e) (void)hipEventDestroy(e);
            delete sl;
        }
        if (had) (void)hipSetDevice(prev);  // the caller's current device is left as it was
    }
    hipError_t take(bool timed, StageSlot** out) {
        std::lock_guard<std::mutex> lk(mu);
        if (free_slots.empty()) {
            StageSlot* sl = new (std::nothrow) StageSlot();
            if (!sl) return hipErrorOutOfMemory;
            hipError_t e = hipMalloc(&sl->mem, slot_bytes);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&sl->after, hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&sl->done, hipEventDisableTiming);
            all.push_back(sl);  // freed with the pool even when incomplete
            if (e != hipSuccess) return e;
            free_slots.push_back(sl);
        }
        StageSlot* sl = free_slots.back();
        if (timed && !sl->tstart) {  // both timed events, or neither
            hipEvent_t a = nullptr, b = nullptr;
            hipError_t e = hipEventCreate(&a);
            if (e == hipSuccess) e = hipEventCreate(&b);
            if (e != hipSuccess) {
                if (a) (void)hipEventDestroy(a);
                return e;
            }
            sl->tstart = a;
            sl->tdone = b;
        }
        free_slots.pop_back();
        *out = sl;
        return hipSuccess;
    }
    void give(StageSlot* sl) {
        std::lock_guard<std::mutex> lk(mu);
        free_slots.push_back(sl);
    }
};

// Environment knobs of a context, read once in ocean_create ("Environment knobs";
// tests/test_abi.py checks that this is every getenv of the library).  The defaults are the measured
// best; every knob changes the schedule only, never the arithmetic of a texel, except OCEAN_Q and
// OCEAN_A4, which select the reference's four-plane passes (within the fp32 tolerance / bit-identical).
struct ocean_options {
    int q = 1;              // OCEAN_Q=0: the four-plane fused frame where the three-plane one applies
    int a4 = 1;             // OCEAN_A4=0: the per-texel row pass A3 instead of the mirror-pair pass A4
    long chunk_mib = 192;   // OCEAN_CHUNK_MIB: intermediate MiB per unit chunk of a frame (0: whole frame)
    int c4_bands = 0;       // OCEAN_C4_BANDS: N >= 2048 column passes per (unit, band); 0 = auto
    long op_chunk_mib = 0;  // OCEAN_OP_CHUNK_MIB: MiB of unit-planes per chunk of ocean_ifft2d (0: auto)
    int tile_w = 0;         // OCEAN_TILE_W: column-tile width of the fused path at N = 128..1024 (0: auto)
    int disp_cached = -1;   // OCEAN_DISP_CACHED: 0 / 1 force pass BQ's DISP store policy (disp_fits_cache); -1 auto

    static ocean_options from_env() {
        ocean_options o;
        if (const char* e = std::getenv("OCEAN_Q")) o.q = std::atoi(e);
        if (const char* e = std::getenv("OCEAN_A4")) o.a4 = std::atoi(e);
        if (const char* e = std::getenv("OCEAN_CHUNK_MIB")) o.chunk_mib = std::max(0L, std::atol(e));
        if (const char* e = std::getenv("OCEAN_C4_BANDS")) o.c4_bands = std::max(0, std::atoi(e));
        if (const char* e = std::getenv("OCEAN_OP_CHUNK_MIB")) o.op_chunk_mib = std::max(0L, std::atol(e));
        if (const char* e = std::getenv("OCEAN_TILE_W")) o.tile_w = std::max(0, std::atoi(e));
        if (const char* e = std::getenv("OCEAN_DISP_CACHED")) o.disp_cached = std::strcmp(e, "auto") ? std::atoi(e) != 0 : -1;
        return o;
    }
};

struct ocean_ctx {
    int device = 0;
    int n = 0, logn = 0, C = 0, T = 0, P = 4;
    uint32_t flags = 0;
    hipStream_t stream = nullptr;
    // device buffers
    float2* noise = nullptr;
    float4* h0 = nullptr;
    float2* h0k = nullptr;   // h0.xy for the mirror-pair row passes: pass_a4_supported sizes, and pass A3PP
                             // at N = 4096 (allocated by ocean_set_column_parity)
    bool h0k_valid = false;  // h0k matches h0 (false after ocean_write(H0): .zw may then be arbitrary)
    bool h0_conj = false;    // h0.zw = conj h0(-k) (from ocean_init_spectrum; the three-plane frame needs it)
    ocean_options opt;       // environment knobs, read once in ocean_create
    size_t inter_units = 0;  // units the intermediate holds (one chunk of a frame; every chunk reuses it)
    int band_x0 = 0, band_nx = 0;  // column band of the fused passes (ocean_set_column_band); nx = n: whole
    int col_par = -1;              // column parity (ocean_set_column_parity): -1 off, else x = 2 m + col_par
    int tile_w = 8;                // column-tile width of the fused path's tile-major layouts (ocean_create)
    float4* waves = nullptr;
    float2* plane[4] = {nullptr, nullptr, nullptr, nullptr};
    float4* disp = nullptr;
    float4* deriv = nullptr;
    float4* turb = nullptr;
    float4* normal = nullptr;
    float2* tw = nullptr;
    float* casc = nullptr;
    float2* tplane = nullptr;  // fused-path intermediate (tile-major), P planes
    float* foam = nullptr;     // foam state (tile-major)
    float2* qside = nullptr;   // three-plane frame side arrays (d0, srow per unit of a chunk)
    float4* deriv_mips = nullptr;  // OCEAN_F_MIPS chains (levels 1..log2 N per slice)
    float4* turb_mips = nullptr;
    size_t mip_chain = 0;
    hipStream_t copy_stream = nullptr;  // ocean_read_async / ocean_read_height_async
    std::shared_ptr<StagePool> stage_pool;  // their staging slots
    bool readback_timing = false;           // ocean_set_readback_timing
    // host state.  `params` and the device `casc` are what the kernels run with; set_params
    // only stages new values, which ocean_init_spectrum makes active (ocean.h), so a
    // frame stepped between the two still uses the spectrum's own constants.
    ocean::SpectrumParams params{};
    ocean::SpectrumParams staged_params{};
    float staged_casc[5 * ocean::kMaxCascades] = {};
    bool params_set = false;
    std::vector<bool> noise_set;
    bool spectrum_ready = false;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> event_pool;
    std::vector<TimedLaunch> pending;
    double kind_ms[3] = {0, 0, 0};
    long long kind_count[3] = {0, 0, 0};
    const void* kind_kernel[3] = {nullptr, nullptr, nullptr};  // last kernel launched per kind (ocean_kernel_name)
    static constexpr size_t kMaxPending = 2048;  // timed launches held before folding into kind_ms

    size_t texels() const { return (size_t)n * n; }
    size_t units() const { return (size_t)T * C; }

    ocean::DevView view() const {
        ocean::DevView v{};
        v.n = n;
        v.logn = logn;
        v.C = C;
        v.T = T;
        v.units = T * C;
        v.planes = P;
        v.normals = (flags & OCEAN_F_NORMALS) != 0;
        v.noise = noise;
        v.h0 = h0;
        v.h0k = h0k;
        v.waves = waves;
        for (int p = 0; p < 4; ++p) v.plane[p] = plane[p];
        v.plane_stride = texels() * units();
        v.inter_stride = texels() * inter_units;
        v.disp = disp;
        v.deriv = deriv;
        v.turb = turb;
        v.normal = normal;
        v.tw = tw;
        v.casc = casc;
        v.gravity = params.gravity;
        v.tile_w = tile_w;
        v.tplane = tplane;
        v.foam = foam;
        v.qside = qside;
        v.deriv_mips = deriv_mips;
        v.turb_mips = turb_mips;
        v.mip_chain = mip_chain;
        v.x0 = band_x0;
        v.nx = band_nx;
        v.xstr = col_par >= 0 ? 2 : 1;
        v.xpar = col_par >= 0 ? col_par : 0;
        return v;
    }

    hipEvent_t take_event() {
        if (event_pool.empty()) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            return e;
        }
        hipEvent_t e = event_pool.back();
        event_pool.pop_back();
        return e;
    }
};

namespace {

// The device rule of every entry point (device_scope.h) over the HIP runtime: hipSetDevice only when the
// device differs, and a failure to set it becomes the call's OCEAN_E_DEVICE.
struct HipDeviceApi {
    static int get(int* device) { return (int)hipGetDevice(device); }
    static int set(int device) { return (int)hipSetDevice(device); }
};
class DeviceScope : public ocean::BasicDeviceScope<HipDeviceApi> {
  public:
    explicit DeviceScope(int device) : ocean::BasicDeviceScope<HipDeviceApi>(device) {
        if (error()) status_ = hip_fail((hipError_t)error(), "hipSetDevice");
    }
    int status() const { return status_; }

  private:
    int status_ = OCEAN_OK;
};

}  // namespace

// Entry of every call that touches the device: check the context, make its device current until the
// call returns (DeviceScope), or return the failure.
#define OCEAN_ENTER(ctx)                                                        \
    if (!(ctx)) return fail(OCEAN_E_INVALID_ARG, "null context");              \
    DeviceScope device_scope_((ctx)->device);                                   \
    if (const int device_scope_status_ = device_scope_.status()) return device_scope_status_

namespace {

// Folds timed launches into kind_ms / kind_count and returns their events to the pool.
// wait: synchronize the stream first (every pending launch is then finished); else fold
// the finished prefix only (stream order: the first unfinished launch ends it).
int fold_pending(ocean_ctx* ctx, bool wait) {
    if (wait) OCEAN_HIP(hipStreamSynchronize(ctx->stream));
    size_t k = 0;
    for (; k < ctx->pending.size(); ++k) {
        const TimedLaunch& t = ctx->pending[k];
        if (!wait) {
            const hipError_t q = hipEventQuery(t.b);
            if (q == hipErrorNotReady) break;
            if (q != hipSuccess) return hip_fail(q, "hipEventQuery");
        }
        float ms = 0.0f;
        OCEAN_HIP(hipEventElapsedTime(&ms, t.a, t.b));
        ctx->kind_ms[t.kind] += ms;
        ctx->kind_count[t.kind] += 1;
        ctx->event_pool.push_back(t.a);
        ctx->event_pool.push_back(t.b);
    }
    ctx->pending.erase(ctx->pending.begin(), ctx->pending.begin() + k);
    return OCEAN_OK;
}

// Launch wrapper: when kernel timing is on, the kernels launched by `launch` carry an event
// pair (ocean_internal.h, launch_events).  A host that never polls ocean_kernel_stats holds
// at most kMaxPending launches' events.
template <class F>
int timed(ocean_ctx* ctx, int kind, F&& launch, const char* what) {
    ocean::last_kernel() = nullptr;
    if (!ctx->timing) {
        const hipError_t e = launch();
        if (ocean::last_kernel()) ctx->kind_kernel[kind] = ocean::last_kernel();
        return e == hipSuccess ? OCEAN_OK : hip_fail(e, what);
    }
    if (ctx->pending.size() >= ocean_ctx::kMaxPending) {
        if (int r = fold_pending(ctx, false)) return r;
        if (ctx->pending.size() >= ocean_ctx::kMaxPending)
            if (int r = fold_pending(ctx, true)) return r;
    }
    ocean::LaunchEvents ev{ctx->take_event(), ctx->take_event(), false};
    if (!ev.start || !ev.stop) return fail(OCEAN_E_DEVICE, "hipEventCreate failed");
    ocean::launch_events() = &ev;  // the kernels of this entry carry the events (ocean_internal.h)
    const hipError_t e = launch();
    ocean::launch_events() = nullptr;
    if (ocean::last_kernel()) ctx->kind_kernel[kind] = ocean::last_kernel();
    if (e != hipSuccess) return hip_fail(e, what);
    if (!ev.launched) {  // nothing was launched: an empty interval
        OCEAN_HIP(hipEventRecord(ev.start, ctx->stream));
        OCEAN_HIP(hipEventRecord(ev.stop, ctx->stream));
    }
    ctx->pending.push_back({kind, ev.start, ev.stop});
    return OCEAN_OK;
}

void* tex_ptr(ocean_ctx* ctx, int tex, size_t* elem_bytes, size_t* slices) {
    *slices = ctx->units();
    switch (tex) {
        case OCEAN_TEX_NOISE: *elem_bytes = 8; *slices = ctx->T; return ctx->noise;
        case OCEAN_TEX_H0: *elem_bytes = 16; return ctx->h0;
        case OCEAN_TEX_WAVES: *elem_bytes = 16; return ctx->waves;
        case OCEAN_TEX_PLANE0:
        case OCEAN_TEX_PLANE1:
        case OCEAN_TEX_PLANE2:
        case OCEAN_TEX_PLANE3: *elem_bytes = 8; return ctx->plane[tex - OCEAN_TEX_PLANE0];
        case OCEAN_TEX_DISP: *elem_bytes = 16; return ctx->disp;
        case OCEAN_TEX_DERIV: *elem_bytes = 16; return ctx->deriv;
        case OCEAN_TEX_TURB: *elem_bytes = 16; return ctx->turb;
        case OCEAN_TEX_NORMAL: *elem_bytes = 16; return ctx->normal;
    }
    return nullptr;
}

int slice_ptr(ocean_ctx* ctx, int tex, int tile, int cascade, size_t bytes, char** out) {
    size_t eb = 0, slices = 0;
    void* base = tex_ptr(ctx, tex, &eb, &slices);
    if (tex < OCEAN_TEX_NOISE || tex > OCEAN_TEX_NORMAL) return fail(OCEAN_E_INVALID_ARG, "unknown texture id");
    if (!base) return fail(OCEAN_E_INVALID_ARG, "texture not allocated for this context's flags");
    if (tile < 0 || tile >= ctx->T) return fail(OCEAN_E_INVALID_ARG, "tile out of range");
    if (tex != OCEAN_TEX_NOISE && (cascade < 0 || cascade >= ctx->C))
        return fail(OCEAN_E_INVALID_ARG, "cascade out of range");
    const size_t slice_bytes = ctx->texels() * eb;
    if (bytes != slice_bytes)
        return fail(OCEAN_E_INVALID_ARG, "byte count " + std::to_string(bytes) + " != slice size " +
                                             std::to_string(slice_bytes));
    const size_t slice = tex == OCEAN_TEX_NOISE ? (size_t)tile : (size_t)tile * ctx->C + cascade;
    *out = static_cast<char*>(base) + slice * slice_bytes;
    return OCEAN_OK;
}

void free_all(ocean_ctx* c) {
    void* ptrs[] = {c->noise, c->h0, c->h0k, c->waves, c->plane[0], c->disp, c->deriv,
                    c->turb,  c->normal, c->tw,    c->casc,     c->tplane, c->foam, c->deriv_mips, c->turb_mips,
                    c->qside};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (auto& t : c->pending) {
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    for (auto e : c->event_pool) (void)hipEventDestroy(e);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    if (c->stream) (void)hipStreamDestroy(c->stream);
}

}  // namespace

namespace {
int chunk_units(const ocean_ctx* ctx, int planes);
// intermediate planes of the three-plane frame: Q1..Q3, plus the four-step column passes' R[Q4]
int q_planes(const ocean_ctx* ctx) { return ctx->n >= 2048 ? 4 : 3; }
}  // namespace

extern "C" {

const char* ocean_last_error(void) { return g_last_error.c_str(); }

int ocean_abi_version(void) { return OCEAN_ABI_VERSION; }

int ocean_create(int device, int n, int n_cascades, int n_tiles, uint32_t flags, ocean_ctx** out) {
    g_last_error.clear();
    if (!out) return fail(OCEAN_E_INVALID_ARG, "out is null");
    *out = nullptr;
    if (n < 16 || n > 4096 || (n & (n - 1)) != 0)
        return fail(OCEAN_E_UNSUPPORTED, "n must be a power of two in [16, 4096], got " + std::to_string(n));
    if (n_cascades < 1 || n_cascades > ocean::kMaxCascades)
        return fail(OCEAN_E_UNSUPPORTED, "n_cascades must be in [1, 5], got " + std::to_string(n_cascades));
    if (n_tiles < 1) return fail(OCEAN_E_INVALID_ARG, "n_tiles must be >= 1");
    if (flags & ~(OCEAN_F_DISPLACEMENT_ONLY | OCEAN_F_NORMALS | OCEAN_F_UNFUSED | OCEAN_F_MIPS))
        return fail(OCEAN_E_INVALID_ARG, "unknown flag bits");
    if ((flags & OCEAN_F_DISPLACEMENT_ONLY) && (flags & OCEAN_F_NORMALS))
        return fail(OCEAN_E_INVALID_ARG, "NORMALS needs the derivative planes (not DISPLACEMENT_ONLY)");
    if ((flags & OCEAN_F_DISPLACEMENT_ONLY) && (flags & OCEAN_F_MIPS))
        return fail(OCEAN_E_INVALID_ARG, "MIPS chains are on DERIV and TURB (not DISPLACEMENT_ONLY)");
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    if (device < 0 || device >= ndev) return fail(OCEAN_E_INVALID_ARG, "device index out of range");
    DeviceScope device_scope(device);  // the caller's current device is restored on return
    if (const int r = device_scope.status()) return r;

    ocean_ctx* c = new (std::nothrow) ocean_ctx();
    if (!c) return fail(OCEAN_E_OUT_OF_MEMORY, "host allocation failed");
    c->device = device;
    c->n = n;
    c->logn = 0;
    while ((1 << c->logn) < n) c->logn++;
    c->C = n_cascades;
    c->T = n_tiles;
    c->flags = flags;
    c->P = (flags & OCEAN_F_DISPLACEMENT_ONLY) ? 2 : 4;
    c->noise_set.assign(n_tiles, false);
    c->band_nx = n;
    c->opt = ocean_options::from_env();
    // Width of the fused path's column tiles.  With fewer tiles than CUs (one 512^2
    // cascade: 32 tiles of 16 columns) pass B ran on an eighth of the chip, so small
    // jobs at N <= 512 take 4-column tiles (docs/MEASUREMENTS.md section 3; at N = 1024 pass A's
    // 32-byte tile rows cost what pass B gains).  OCEAN_TILE_W overrides (A/B).
    c->tile_w = ocean::fftcore::inter_w(n);
    {
        int cus = 256;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
            cus = 256;
        const long tiles = (long)n_cascades * n_tiles * (n / c->tile_w);
        if (n >= 128 && n <= 512 && tiles < cus) c->tile_w = 4;
        const int w = c->opt.tile_w;
        if (w && n >= 128 && n <= 1024 && (w == 4 || w == ocean::fftcore::inter_w(n))) c->tile_w = w;
    }

    auto alloc = [&](void** p, size_t bytes) -> bool {
        if (hipMalloc(p, bytes) != hipSuccess) return false;
        return hipMemset(*p, 0, bytes) == hipSuccess;
    };
    const size_t tex = c->texels(), U = c->units();
    bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && alloc((void**)&c->noise, tex * c->T * 8);
    ok = ok && alloc((void**)&c->h0, tex * U * 16);
    // h0k: the mirror-pair row passes (N = 256 / 512 / 1024; at 4096 the column-parity pass A3PP allocates
    // it in ocean_set_column_parity)
    if (ocean::pass_a4_supported(n, c->P)) ok = ok && alloc((void**)&c->h0k, tex * U * 8);
    ok = ok && alloc((void**)&c->waves, tex * U * 16);
    ok = ok && alloc((void**)&c->plane[0], tex * U * 8 * c->P);  // planes contiguous (one descriptor in pass A)
    if (ok)
        for (int p = 1; p < c->P; ++p) c->plane[p] = c->plane[0] + (size_t)p * tex * U;
    ok = ok && alloc((void**)&c->disp, tex * U * 16);
    if (c->P == 4) {
        ok = ok && alloc((void**)&c->deriv, tex * U * 16);
        ok = ok && alloc((void**)&c->turb, tex * U * 16);
        ok = ok && alloc((void**)&c->foam, tex * U * 4);
    }
    // the intermediate holds a chunk of either schedule: P planes, or (three-plane frame) planes
    // Q1..Q3 plus the per-unit side arrays in the fourth plane's room (fftq.hip)
    c->inter_units = (size_t)std::max(chunk_units(c, c->P),
                                      ocean::pass_q_supported(n, c->P) ? chunk_units(c, q_planes(c)) : 1);
    ok = ok && alloc((void**)&c->tplane, tex * c->inter_units * 8 * c->P);
    if (ocean::pass_q_supported(n, c->P)) ok = ok && alloc((void**)&c->qside, c->inter_units * 2 * n * 8);
    if (flags & OCEAN_F_NORMALS) ok = ok && alloc((void**)&c->normal, tex * U * 16);
    if (flags & OCEAN_F_MIPS) {
        for (int l = 1; (n >> l) >= 1; ++l) c->mip_chain += (size_t)(n >> l) * (n >> l);
        ok = ok && alloc((void**)&c->deriv_mips, c->mip_chain * U * 16);
        ok = ok && alloc((void**)&c->turb_mips, c->mip_chain * U * 16);
    }
    const size_t tw_entries = (size_t)n + 128 + ocean::stage_twiddle_entries(n);
    ok = ok && alloc((void**)&c->tw, tw_entries * 8);
    ok = ok && alloc((void**)&c->casc, 5 * 4 * 5);
    if (!ok) {
        std::string msg = std::string("device allocation failed: ") + hipGetErrorString(hipGetLastError());
        free_all(c);
        delete c;
        return fail(OCEAN_E_OUT_OF_MEMORY, msg);
    }
    // twiddle table tw[m] = exp(+2 pi i m / N), double precision then rounded
    std::vector<float2> tw(tw_entries);
    for (int m = 0; m < n; ++m) {
        const double a = 2.0 * M_PI * (double)m / (double)n;
        tw[m] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    for (int k = 0; k < 64; ++k) {
        const double lo = 2.0 * M_PI * (double)k / (double)n, hi = 2.0 * M_PI * 64.0 * (double)k / (double)n;
        tw[n + k] = make_float2((float)std::cos(lo), (float)std::sin(lo));
        tw[n + 64 + k] = make_float2((float)std::cos(hi), (float)std::sin(hi));
    }
    // per-stage tables for the plans with first radix 16, 8 and 4 (fft_engine.h StageTw):
    // stage s >= 1 (Ns, R), entry r*Ns + k = exp(+2 pi i r k / (Ns R))
    {
        using namespace ocean::fftcore;
        size_t o = (size_t)n + 128;
        for (int r0 : {16, 8, 4})
            for (int s = 1; s < n_stages(n, r0); ++s) {
                const int ns = ns_of(n, s, r0), r = radix_of(n, s, r0);
                for (int q = 0; q < r; ++q)
                    for (int k = 0; k < ns; ++k) {
                        const double a = 2.0 * M_PI * (double)q * (double)k / ((double)ns * (double)r);
                        tw[o++] = make_float2((float)std::cos(a), (float)std::sin(a));
                    }
            }
    }
    e = hipMemcpy(c->tw, tw.data(), tw_entries * 8, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        free_all(c);
        delete c;
        return hip_fail(e, "twiddle upload");
    }
    *out = c;
    return OCEAN_OK;
}

void ocean_destroy(ocean_ctx* ctx) {
    if (!ctx) return;
    DeviceScope device_scope(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    free_all(ctx);
    delete ctx;
}

int ocean_set_params(ocean_ctx* ctx, const ocean_params* params, const ocean_cascade* cascades) {
    OCEAN_ENTER(ctx);
    if (!params || !cascades) return fail(OCEAN_E_INVALID_ARG, "null params/cascades");
    const ocean_params& p = *params;
    if (!(p.gravity > 0) || !(p.fetch > 0) || !(p.wind_speed > 0) || !std::isfinite(p.depth))
        return fail(OCEAN_E_INVALID_ARG, "gravity, fetch and wind_speed must be > 0, depth finite");
    if (p.wind_dir_x == 0.0f && p.wind_dir_y == 0.0f) return fail(OCEAN_E_INVALID_ARG, "zero wind direction");
    float h[25];
    for (int c = 0; c < ctx->C; ++c) {
        const ocean_cascade& k = cascades[c];
        if (!(k.wavelength > 0)) return fail(OCEAN_E_INVALID_ARG, "cascade wavelength must be > 0");
        h[c * 5 + 0] = k.wavelength;
        h[c * 5 + 1] = k.cutoff_low;
        h[c * 5 + 2] = k.cutoff_high;
        h[c * 5 + 3] = k.swell;
        h[c * 5 + 4] = k.fade;
    }
    // staged only: the running spectrum (h0, and the wave data the fused row pass rebuilds
    // every frame from casc + gravity) keeps its constants until ocean_init_spectrum
    std::memcpy(ctx->staged_casc, h, sizeof(float) * 5 * ctx->C);
    ctx->staged_params = {p.wind_speed, p.wind_dir_x, p.wind_dir_y, p.gravity, p.fetch, p.depth};
    ctx->params_set = true;
    return OCEAN_OK;
}

int ocean_set_noise(ocean_ctx* ctx, int tile, const float* rg) {
    OCEAN_ENTER(ctx);
    if (!rg) return fail(OCEAN_E_INVALID_ARG, "null noise");
    char* dst = nullptr;
    if (int r = slice_ptr(ctx, OCEAN_TEX_NOISE, tile, 0, ctx->texels() * 8, &dst)) return r;
    OCEAN_HIP(hipMemcpyAsync(dst, rg, ctx->texels() * 8, hipMemcpyHostToDevice, ctx->stream));
    OCEAN_HIP(hipStreamSynchronize(ctx->stream));
    ctx->noise_set[tile] = true;
    return OCEAN_OK;
}

int ocean_generate_noise_device(ocean_ctx* ctx, uint64_t seed) {
    OCEAN_ENTER(ctx);
    const ocean::DevView v = ctx->view();
    OCEAN_HIP(ocean::launch_noise(v, seed, ctx->stream));
    OCEAN_HIP(hipStreamSynchronize(ctx->stream));
    for (int t = 0; t < ctx->T; ++t) ctx->noise_set[t] = true;
    return OCEAN_OK;
}

int ocean_generate_noise(ocean_ctx* ctx, uint64_t seed) {
    OCEAN_ENTER(ctx);
    std::vector<float> host(ctx->texels() * 2);
    for (int t = 0; t < ctx->T; ++t) {
        ocean::generate_noise_host(ctx->n, seed + (uint64_t)t, host.data());
        if (int r = ocean_set_noise(ctx, t, host.data())) return r;
    }
    return OCEAN_OK;
}

int ocean_init_spectrum(ocean_ctx* ctx) {
    OCEAN_ENTER(ctx);
    if (!ctx->params_set) return fail(OCEAN_E_STATE, "ocean_set_params must precede ocean_init_spectrum");
    for (int t = 0; t < ctx->T; ++t)
        if (!ctx->noise_set[t]) return fail(OCEAN_E_STATE, "noise not set for tile " + std::to_string(t));
    // the staged parameters become active (stream-ordered: frames queued before this
    // call still read the previous constants)
    OCEAN_HIP(hipMemcpyAsync(ctx->casc, ctx->staged_casc, (size_t)ctx->C * 5 * 4, hipMemcpyHostToDevice, ctx->stream));
    OCEAN_HIP(hipStreamSynchronize(ctx->stream));
    ctx->params = ctx->staged_params;
    const ocean::DevView v = ctx->view();
    if (int r = timed(ctx, 2, [&] { return ocean::launch_init_spectrum(v, ctx->params, ctx->stream); },
                      "init_spectrum"))
        return r;
    if (int r = timed(ctx, 2, [&] { return ocean::launch_conjugate(v, ctx->stream); }, "conjugate")) return r;
    // the foam state is left alone: the reference re-runs CalculateInitialSpectrumTextures on a
    // parameter change (the commented OnValidate, WaterBody.cs:324-337) without touching
    // _TurbulenceTextures; it starts at zero (ocean_create) and ocean_reset_foam clears it
    ctx->spectrum_ready = true;
    ctx->h0k_valid = ctx->h0k != nullptr;
    ctx->h0_conj = true;
    return OCEAN_OK;
}

int ocean_reset_foam(ocean_ctx* ctx) {
    OCEAN_ENTER(ctx);
    if (ctx->turb) OCEAN_HIP(hipMemsetAsync(ctx->turb, 0, ctx->texels() * ctx->units() * 16, ctx->stream));
    if (ctx->foam) OCEAN_HIP(hipMemsetAsync(ctx->foam, 0, ctx->texels() * ctx->units() * 4, ctx->stream));
    if (ctx->turb_mips) OCEAN_HIP(hipMemsetAsync(ctx->turb_mips, 0, ctx->mip_chain * ctx->units() * 16, ctx->stream));
    return OCEAN_OK;
}

int ocean_evolve(ocean_ctx* ctx, float time) {
    OCEAN_ENTER(ctx);
    if (!ctx->spectrum_ready) return fail(OCEAN_E_STATE, "ocean_init_spectrum must precede ocean_evolve");
    const ocean::DevView v = ctx->view();
    return timed(ctx, 2, [&] { return ocean::launch_evolve(v, time, ctx->stream); }, "evolve");
}

int ocean_ifft2d(ocean_ctx* ctx, int plane_mask) {
    OCEAN_ENTER(ctx);
    if (plane_mask < 0 || plane_mask > 15) return fail(OCEAN_E_INVALID_ARG, "plane_mask must be in [0, 15]");
    for (int p = 0; p < 4; ++p)
        if ((plane_mask & (1 << p)) && p >= ctx->P)
            return fail(OCEAN_E_INVALID_ARG, "plane not allocated (DISPLACEMENT_ONLY context)");
    const ocean::DevView v = ctx->view();
    const size_t up_elems = ctx->texels();  // one unit-plane
    for (int p = 0; p < 4;) {
        if (!(plane_mask & (1 << p))) {
            ++p;
            continue;
        }
        int np = 1;  // run of consecutive planes: one launch per direction (planes are one allocation)
        while (p + np < 4 && (plane_mask & (1 << (p + np)))) ++np;
        if (ctx->n == 4096) {
            // Folded columns, in place (fft2.hip k_rowsf / k_colsf_ip): per chunk of unit-planes, rows +
            // the decimation-in-frequency fold onto the planes' own rows (z_b at rows b L + n), then
            // 2048-point column tiles of both sub-planes per item, back into the planes, permuted.  A chunk
            // of at most OCEAN_OP_CHUNK_MIB stays in the Infinity Cache between the two launches (auto 256
            // MiB: two unit-planes; docs/MEASUREMENTS.md section 8).
            const int ups = np * (int)ctx->units();
            const long mib = ctx->opt.op_chunk_mib > 0 ? ctx->opt.op_chunk_mib : 256;
            const int k = (int)std::max<size_t>(1, ((size_t)mib << 20) / (up_elems * 8));
            for (int c0 = 0; c0 < ups; c0 += k) {
                const int kc = std::min(k, ups - c0);
                float2* planes = ctx->plane[p] + (size_t)c0 * up_elems;
                if (int r = timed(ctx, 0, [&] { return ocean::launch_ifft_fold(v, planes, kc, 0, ctx->stream); },
                                  "ifft_rows"))
                    return r;
                if (int r = timed(ctx, 1, [&] { return ocean::launch_ifft_fold(v, planes, kc, 1, ctx->stream); },
                                  "ifft_cols"))
                    return r;
            }
            p += np;
            continue;
        }
        // In-place row and column launches per chunk of at most OCEAN_OP_CHUNK_MIB of unit-planes, so
        // the column launch re-reads the rows' output from the Infinity Cache when the plane set is
        // larger than it.  Auto: 256 MiB (4 x 4 x 1024^2 x 4 planes, 512 MiB, fresh data: 128 / 192 /
        // 256 / 320 / 384 MiB / unchunked 0.69 / 0.69 / 0.736 / 0.63 / 0.60 / 0.57 of peak; cfg3's 128
        // MiB: one chunk).  At N = 1024 / 2048 the column launch takes XCD-paired halves of 16-column
        // tiles (fft2.hip Cols2).
        const int ups = np * (int)ctx->units();
        const long mib = ctx->opt.op_chunk_mib > 0 ? ctx->opt.op_chunk_mib : 256;
        const int k = (int)std::max<size_t>(1, ((size_t)mib << 20) / (up_elems * 8));
        for (int c0 = 0; c0 < ups; c0 += k) {
            const int kc = std::min(k, ups - c0);
            float2* base = ctx->plane[p] + (size_t)c0 * up_elems;
            if (int r = timed(ctx, 0, [&] { return ocean::launch_ifft_rows_v2(v, base, kc, ctx->stream); }, "ifft_rows"))
                return r;
            if (int r = timed(ctx, 1, [&] { return ocean::launch_ifft_cols_v2(v, base, kc, ctx->stream); }, "ifft_cols"))
                return r;
        }
        p += np;
    }
    return OCEAN_OK;
}

int ocean_fill(ocean_ctx* ctx) {
    OCEAN_ENTER(ctx);
    const ocean::DevView v = ctx->view();
    return timed(ctx, 2, [&] { return ocean::launch_fill(v, ctx->stream); }, "fill");
}

namespace {
int step_fused(ocean_ctx* ctx, float time);
bool use_q(const ocean_ctx* ctx);

// GenerateMips (WaterBody.cs:191-192) when the context has mip chains.
int generate_mips(ocean_ctx* ctx) {
    if (!(ctx->flags & OCEAN_F_MIPS)) return OCEAN_OK;
    const ocean::DevView v = ctx->view();
    return timed(ctx, 2, [&] { return ocean::launch_mips(v, ctx->stream); }, "mips");
}
}  // namespace

int ocean_step(ocean_ctx* ctx, float time) {
    OCEAN_ENTER(ctx);
    if (!ctx->spectrum_ready) return fail(OCEAN_E_STATE, "ocean_init_spectrum must precede ocean_step");
    if (ctx->flags & OCEAN_F_UNFUSED) {
        if (int r = ocean_evolve(ctx, time)) return r;
        if (int r = ocean_ifft2d(ctx, (1 << ctx->P) - 1)) return r;
        if (int r = ocean_fill(ctx)) return r;
        return generate_mips(ctx);
    }
    if (int r = step_fused(ctx, time)) return r;
    return generate_mips(ctx);
}

namespace {
// View of units [u0, u0 + nu) (unit u of the view is cascade (c0 + u) % C).
ocean::DevView sub_view(const ocean::DevView& v, int u0, int nu, bool inter_at_base = false) {
    ocean::DevView s = v;
    const size_t off = (size_t)u0 * v.n * v.n;
    s.units = nu;
    s.c0 = (v.c0 + u0) % v.C;
    s.h0 = v.h0 + off;
    s.waves = v.waves + off;
    if (v.h0k) s.h0k = v.h0k + off;
    // plane_stride unchanged: planes stay U * N * N apart.  inter_at_base: the chunk's
    // intermediate starts at the base of every plane (one region reused by every chunk)
    s.tplane = inter_at_base ? v.tplane : v.tplane + off;
    if (v.foam) s.foam = v.foam + off;
    if (v.qside) s.qside = inter_at_base ? v.qside : v.qside + (size_t)u0 * 2 * v.n;
    s.disp = v.disp + off;
    if (v.deriv) s.deriv = v.deriv + off;
    if (v.turb) s.turb = v.turb + off;
    if (v.normal) s.normal = v.normal + off;
    return s;
}

// Units per chunk: a frame over many units runs pass A and pass B chunk by chunk so
// that the intermediate pass B re-reads is still in the 256 MiB Infinity Cache
// (OCEAN_CHUNK_MIB of intermediate per chunk, 0 = whole frame at once; a unit larger than a
// chunk: whole frame).  Measured on cfg4's 1024 units at 512^2 (8 MiB each): 64 MiB 37.9k,
// 128 MiB 40.7k, 192 MiB 43.1k, 256 MiB 38.4k, unchunked 40.7k tile-frames/s.
int chunk_units(const ocean_ctx* ctx, int planes) {
    const long mib = ctx->opt.chunk_mib;
    const int U = (int)ctx->units();
    if (mib <= 0) return U;
    const size_t per_unit = ctx->texels() * 8 * planes;
    int k = (int)(((size_t)mib << 20) / per_unit);
    if (k >= ctx->C) k -= k % ctx->C;  // whole tiles when a chunk holds one
    if (k < 1) return U;
    return k >= U ? U : k;
}

// Column bands per unit for the N >= 2048 column passes: OCEAN_C4_BANDS, or by default
// as many as keep one band's planes (P * N * width * 8 B) within 256 MiB -- cfg5's 512 MiB
// units run as 2 bands: 387 -> 412-421 frames/s (3 or 4 bands: 417; per-unit pass A: slower).
// Band widths stay multiples of the four-step tile width (16).
int c4_bands(const ocean_ctx* ctx, int nx) {
    if (!ocean::pass_c4_supported(ctx->n)) return 1;
    int nb = ctx->opt.c4_bands;
    if (nb <= 0) {
        const size_t band_bytes = (size_t)ctx->P * ctx->n * nx * 8;
        nb = 1;
        while (band_bytes / nb > ((size_t)256 << 20)) nb *= 2;
    }
    while (nb > 1 && (nx % nb || (nx / nb) % 16)) --nb;
    return nb;
}

// The three-plane fused frame (fftq.hip) runs where it applies: N = 512 / 1024 with full
// outputs, the mirror-pair row pass's h0k valid.
bool use_q(const ocean_ctx* ctx) {
    if (!ctx->opt.q || !ctx->h0_conj || !ocean::pass_q_supported(ctx->n, ctx->P)) return false;
    return ctx->n >= 2048 || (ctx->opt.a4 && ctx->h0k_valid);  // N <= 1024: the mirror-pair row pass reads h0k
}

// Pass BQ may write DISP with default-policy stores (DevView::disp_cached) when the whole frame is one chunk
// and its cache-resident set plus DISP fits 224 MiB of the 256 MiB Infinity Cache of an MI355X: DISP then
// waits there and is written back while the next pass A runs, when HBM has headroom.  The resident set is
// what the three-plane frame re-reads each frame, per texel-cascade: pass AQ's h0k (8 B; the frame runs
// only with the mirror-pair row pass, use_q), the intermediate Q1..Q3 (24 B) and the foam state (4 B).
// cfg3 (4 x 1024^2, 208 MiB): 11.83-11.88 -> 12.08-12.11 k frames/s; a cfg4 chunk (32 units of 512^2,
// 288 MiB) lost 7.5 % the same way, and DISP + TURB at cfg3 lost 7 % (docs/MEASUREMENTS.md section 8).
// The 224 MiB budget is this part's; OCEAN_DISP_CACHED=0 / 1 overrides the choice (A/B, other parts).
bool disp_fits_cache(const ocean_ctx* ctx, bool q, int chunk) {
    if (!q || ctx->n > 1024 || chunk < (int)ctx->units()) return false;
    if (ctx->opt.disp_cached >= 0) return ctx->opt.disp_cached != 0;
    constexpr size_t kH0k = 8, kInter = 24, kFoam = 4, kDisp = 16;
    const size_t bytes = ctx->texels() * ctx->units() * (kH0k + kInter + kFoam + kDisp);
    return bytes <= ((size_t)224 << 20);
}

int step_fused(ocean_ctx* ctx, float time) {
    // pass A: mirror-pair rows (N = 512, 1024 with 4 planes and h0k valid) or per-texel
    // rows; pass B: column tiles (N <= 1024) or the four-step column passes (N >= 2048)
    ocean::DevView v = ctx->view();
    if (!ctx->h0k_valid) v.h0k = nullptr;  // stale after an H0 upload: no row pass may read it
    const bool q = use_q(ctx);
    if (ctx->col_par >= 0 && !q)
        return fail(OCEAN_E_STATE, "a column parity needs the three-plane frame (h0 from ocean_init_spectrum)");
    const int U = (int)ctx->units(), K = std::min(chunk_units(ctx, q ? q_planes(ctx) : ctx->P), (int)ctx->inter_units);
    v.disp_cached = disp_fits_cache(ctx, q, K);
    for (int u0 = 0; u0 < U; u0 += K) {
        const ocean::DevView c = (K >= U) ? v : sub_view(v, u0, std::min(K, U - u0), ctx->inter_units < ctx->units());
        if (q && ctx->n >= 2048) {
            if (int r = timed(ctx, 0, [&] { return ocean::launch_pass_a_q(c, time, ctx->stream); }, "pass_a")) return r;
            const int nb = c4_bands(ctx, c.nx);
            if (nb == 1) {
                if (int r = timed(ctx, 1, [&] { return ocean::launch_pass_c4q(c, ctx->stream); }, "pass_c")) return r;
                continue;
            }
            const int w = c.nx / nb;
            for (int u = 0; u < c.units; ++u)
                for (int b = 0; b < nb; ++b) {
                    ocean::DevView cb = sub_view(c, u, 1);
                    cb.x0 = c.x0 + b * w;
                    cb.nx = (b == nb - 1) ? c.nx - b * w : w;
                    if (int r = timed(ctx, 1, [&] { return ocean::launch_pass_c4q(cb, ctx->stream); }, "pass_c"))
                        return r;
                }
            continue;
        }
        if (q) {
            if (int r = timed(ctx, 0, [&] { return ocean::launch_pass_a_q(c, time, ctx->stream); }, "pass_a")) return r;
            if (int r = timed(ctx, 1, [&] { return ocean::launch_pass_b_q(c, ctx->stream); }, "pass_b")) return r;
            continue;
        }
        if (int r = timed(ctx, 0, [&] {
                // h0k also exists at 4096 (pass A3PP), where the mirror-pair pass A4 does not
                if (ctx->opt.a4 && ctx->h0k_valid && ocean::pass_a4_supported(ctx->n, ctx->P))
                    return ocean::launch_pass_a_v4(c, time, ctx->stream);
                return ocean::launch_pass_a_v3(c, time, ctx->stream);
            }, "pass_a"))
            return r;
        const int nb = c4_bands(ctx, c.nx);
        if (nb > 1) {
            // four-step column passes per (unit, column band): pass C2 re-reads what C1
            // just wrote while it is still in the Infinity Cache (256 MiB)
            const int w = c.nx / nb;
            for (int u = 0; u < c.units; ++u)
                for (int b = 0; b < nb; ++b) {
                    ocean::DevView cb = sub_view(c, u, 1);
                    cb.x0 = c.x0 + b * w;
                    cb.nx = (b == nb - 1) ? c.nx - b * w : w;
                    if (int r = timed(ctx, 1, [&] { return ocean::launch_pass_c4(cb, ctx->stream); }, "pass_c"))
                        return r;
                }
            continue;
        }
        if (int r = timed(ctx, 1, [&] {
                if (ocean::pass_c4_supported(ctx->n)) return ocean::launch_pass_c4(c, ctx->stream);
                return ocean::launch_pass_b_v3(c, ctx->stream);
            }, "pass_b"))
            return r;
    }
    return OCEAN_OK;
}
}  // namespace

int ocean_read(ocean_ctx* ctx, int texture, int tile, int cascade, void* dst, size_t bytes) {
    OCEAN_ENTER(ctx);
    if (!dst) return fail(OCEAN_E_INVALID_ARG, "null destination");
    char* src = nullptr;
    if (int r = slice_ptr(ctx, texture, tile, cascade, bytes, &src)) return r;
    OCEAN_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    OCEAN_HIP(hipStreamSynchronize(ctx->stream));
    return OCEAN_OK;
}

namespace {
// Level `level` (>= 1) of slice (tile, cascade) of DERIV / TURB's mip chain.
int mip_slice_ptr(ocean_ctx* ctx, int texture, int tile, int cascade, int level, char** out, size_t* bytes) {
    if (!(ctx->flags & OCEAN_F_MIPS)) return fail(OCEAN_E_STATE, "context created without OCEAN_F_MIPS");
    if (texture != OCEAN_TEX_DERIV && texture != OCEAN_TEX_TURB)
        return fail(OCEAN_E_INVALID_ARG, "mip chains exist for OCEAN_TEX_DERIV and OCEAN_TEX_TURB only");
    if (level < 1 || (ctx->n >> level) < 1) return fail(OCEAN_E_INVALID_ARG, "mip level out of range");
    if (tile < 0 || tile >= ctx->T || cascade < 0 || cascade >= ctx->C)
        return fail(OCEAN_E_INVALID_ARG, "tile or cascade out of range");
    size_t off = 0;
    for (int l = 1; l < level; ++l) off += (size_t)(ctx->n >> l) * (ctx->n >> l);
    float4* chain = texture == OCEAN_TEX_DERIV ? ctx->deriv_mips : ctx->turb_mips;
    const size_t slice = (size_t)tile * ctx->C + cascade;
    *out = reinterpret_cast<char*>(chain + slice * ctx->mip_chain + off);
    *bytes = (size_t)(ctx->n >> level) * (ctx->n >> level) * 16;
    return OCEAN_OK;
}
}  // namespace

int ocean_read_mip(ocean_ctx* ctx, int texture, int tile, int cascade, int level, void* dst, size_t bytes) {
    if (level == 0) return ocean_read(ctx, texture, tile, cascade, dst, bytes);
    OCEAN_ENTER(ctx);
    if (!dst) return fail(OCEAN_E_INVALID_ARG, "null destination");
    char* src = nullptr;
    size_t want = 0;
    if (int r = mip_slice_ptr(ctx, texture, tile, cascade, level, &src, &want)) return r;
    if (bytes != want)
        return fail(OCEAN_E_INVALID_ARG, "byte count " + std::to_string(bytes) + " != mip slice size " +
                                             std::to_string(want));
    OCEAN_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    OCEAN_HIP(hipStreamSynchronize(ctx->stream));
    return OCEAN_OK;
}

int ocean_get_mip_ptr(ocean_ctx* ctx, int texture, int level, void** ptr, size_t* slice_stride) {
    if (!ctx || !ptr || !slice_stride) return fail(OCEAN_E_INVALID_ARG, "null argument");
    char* p = nullptr;
    size_t bytes = 0;
    if (int r = mip_slice_ptr(ctx, texture, 0, 0, level, &p, &bytes)) return r;
    *ptr = p;
    *slice_stride = ctx->mip_chain * 16;
    return OCEAN_OK;
}

}  // extern "C"

struct ocean_readback {
    int device = 0;
    bool timed = false;  // made with readback timing on: tstart / tdone recorded
    StageSlot* slot = nullptr;
    std::shared_ptr<StagePool> pool;
    hipEvent_t done() const { return timed ? slot->tdone : slot->done; }
};

namespace {
// The host copy of the readbacks: hipMemcpyDeviceToHost (see docs/MEASUREMENTS.md section 8 for the
// engine the runtime picks)
constexpr hipMemcpyKind kReadbackCopyKind = hipMemcpyDeviceToHost;

// A readback request: `snapshot` enqueues the copy of the wanted bytes into the slot on the ctx stream
// (ordered after the queued steps and before later ones, at HBM speed), then the host copy runs on the
// copy stream, off the ctx stream's path -- snapshot semantics, like a readback in Unity's command stream.
template <class Snapshot>
int start_readback(ocean_ctx* ctx, void* dst, size_t bytes, Snapshot&& snapshot, ocean_readback** out) {
    if (!ctx->copy_stream) OCEAN_HIP(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    if (!ctx->stage_pool) {
        ctx->stage_pool = std::make_shared<StagePool>();
        ctx->stage_pool->device = ctx->device;
        ctx->stage_pool->slot_bytes = ctx->texels() * 16;  // the largest slice (float4 textures)
    }
    ocean_readback* rb = new (std::nothrow) ocean_readback();
    if (!rb) return fail(OCEAN_E_OUT_OF_MEMORY, "host allocation failed");
    rb->device = ctx->device;
    rb->pool = ctx->stage_pool;
    rb->timed = ctx->readback_timing;
    hipError_t e = rb->pool->take(rb->timed, &rb->slot);
    if (e == hipSuccess) e = snapshot(rb->slot->mem);
    if (e == hipSuccess) e = hipEventRecord(rb->slot->after, ctx->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(ctx->copy_stream, rb->slot->after, 0);
    if (e == hipSuccess && rb->timed) e = hipEventRecord(rb->slot->tstart, ctx->copy_stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dst, rb->slot->mem, bytes, kReadbackCopyKind, ctx->copy_stream);
    if (e == hipSuccess) e = hipEventRecord(rb->done(), ctx->copy_stream);
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(ctx->copy_stream);
        (void)hipStreamSynchronize(ctx->stream);
        if (rb->slot) rb->pool->give(rb->slot);
        delete rb;
        return hip_fail(e, "readback request");
    }
    *out = rb;
    return OCEAN_OK;
}
}  // namespace

extern "C" {

int ocean_read_async(ocean_ctx* ctx, int texture, int tile, int cascade, void* dst, size_t bytes,
                     ocean_readback** out) {
    if (!out) return fail(OCEAN_E_INVALID_ARG, "out is null");
    *out = nullptr;
    OCEAN_ENTER(ctx);
    if (!dst) return fail(OCEAN_E_INVALID_ARG, "null destination");
    char* src = nullptr;
    if (int r = slice_ptr(ctx, texture, tile, cascade, bytes, &src)) return r;
    return start_readback(
        ctx, dst, bytes, [&](void* slot) { return hipMemcpyAsync(slot, src, bytes, hipMemcpyDeviceToDevice, ctx->stream); },
        out);
}

int ocean_read_height_async(ocean_ctx* ctx, int tile, int cascade, float* dst, size_t bytes, ocean_readback** out) {
    if (!out) return fail(OCEAN_E_INVALID_ARG, "out is null");
    *out = nullptr;
    OCEAN_ENTER(ctx);
    if (!dst) return fail(OCEAN_E_INVALID_ARG, "null destination");
    if (bytes != ctx->texels() * 4)
        return fail(OCEAN_E_INVALID_ARG, "byte count " + std::to_string(bytes) + " != N * N * 4 = " +
                                             std::to_string(ctx->texels() * 4));
    char* src = nullptr;
    if (int r = slice_ptr(ctx, OCEAN_TEX_DISP, tile, cascade, ctx->texels() * 16, &src)) return r;
    return start_readback(
        ctx, dst, bytes,
        [&](void* slot) {
            return ocean::launch_extract_height(reinterpret_cast<const float4*>(src), static_cast<float*>(slot),
                                                ctx->texels(), ctx->stream);
        },
        out);
}

int ocean_set_readback_timing(ocean_ctx* ctx, int enable) {
    if (!ctx) return fail(OCEAN_E_INVALID_ARG, "null context");
    ctx->readback_timing = enable != 0;
    return OCEAN_OK;
}

int ocean_readback_status(ocean_readback* rb) {
    if (!rb) return fail(OCEAN_E_INVALID_ARG, "null readback");
    const hipError_t e = hipEventQuery(rb->done());
    if (e == hipSuccess) return 1;
    if (e == hipErrorNotReady) return 0;
    return hip_fail(e, "hipEventQuery");
}

int ocean_readback_wait(ocean_readback* rb) {
    if (!rb) return fail(OCEAN_E_INVALID_ARG, "null readback");
    OCEAN_HIP(hipEventSynchronize(rb->done()));
    return OCEAN_OK;
}

void ocean_readback_release(ocean_readback* rb) {
    if (!rb) return;
    {
        DeviceScope device_scope(rb->device);
        (void)hipEventSynchronize(rb->done());  // the slot is free only once its host copy has landed
        rb->pool->give(rb->slot);
    }
    delete rb;
}

int ocean_readback_copy_ms(ocean_readback* rb, float* ms) {
    if (!rb || !ms) return fail(OCEAN_E_INVALID_ARG, "null readback or output");
    if (!rb->timed) return fail(OCEAN_E_STATE, "request made without readback timing (ocean_set_readback_timing)");
    const hipError_t q = hipEventQuery(rb->done());
    if (q == hipErrorNotReady) return fail(OCEAN_E_STATE, "readback still pending");
    if (q != hipSuccess) return hip_fail(q, "hipEventQuery");
    OCEAN_HIP(hipEventElapsedTime(ms, rb->slot->tstart, rb->done()));
    return OCEAN_OK;
}

int ocean_host_alloc(size_t bytes, void** out) {
    if (!out || bytes == 0) return fail(OCEAN_E_INVALID_ARG, "null out or zero size");
    *out = nullptr;
    const hipError_t e = hipHostMalloc(out, bytes, hipHostMallocDefault);
    if (e != hipSuccess) return hip_fail(e, "hipHostMalloc");
    return OCEAN_OK;
}

void ocean_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int ocean_write(ocean_ctx* ctx, int texture, int tile, int cascade, const void* src, size_t bytes) {
    OCEAN_ENTER(ctx);
    if (!src) return fail(OCEAN_E_INVALID_ARG, "null source");
    if (texture == OCEAN_TEX_WAVES && !(ctx->flags & OCEAN_F_UNFUSED))
        return fail(OCEAN_E_UNSUPPORTED, "WAVES is read-only under the fused schedule (its row pass rebuilds the "
                                         "wave data from the parameters every frame); create the context with "
                                         "OCEAN_F_UNFUSED to drive ocean_step from uploaded wave data");
    char* dst = nullptr;
    if (int r = slice_ptr(ctx, texture, tile, cascade, bytes, &dst)) return r;
    OCEAN_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    OCEAN_HIP(hipStreamSynchronize(ctx->stream));
    if (texture == OCEAN_TEX_NOISE) ctx->noise_set[tile] = true;
    if (texture == OCEAN_TEX_H0) {  // the v3 row pass reads h0 (.zw included); the three-plane frame
        ctx->h0k_valid = false;     // needs .zw = conj h0(-k), which an upload need not keep
        ctx->h0_conj = false;
    }
    if (texture == OCEAN_TEX_TURB) {  // foam state follows the uploaded TURB.x (resume)
        const ocean::DevView v = ctx->view();
        OCEAN_HIP(ocean::launch_foam_import(v, ctx->stream));
        OCEAN_HIP(hipStreamSynchronize(ctx->stream));
    }
    return OCEAN_OK;
}

int ocean_get_device_ptr(ocean_ctx* ctx, int texture, void** ptr, size_t* bytes) {
    if (!ctx || !ptr || !bytes) return fail(OCEAN_E_INVALID_ARG, "null argument");
    if (texture < OCEAN_TEX_NOISE || texture > OCEAN_TEX_NORMAL) return fail(OCEAN_E_INVALID_ARG, "unknown texture id");
    size_t eb = 0, slices = 0;
    void* base = tex_ptr(ctx, texture, &eb, &slices);
    if (!base) return fail(OCEAN_E_INVALID_ARG, "texture not allocated for this context's flags");
    *ptr = base;
    *bytes = ctx->texels() * eb * slices;
    return OCEAN_OK;
}

int ocean_get_stream(ocean_ctx* ctx, void** stream) {
    if (!ctx || !stream) return fail(OCEAN_E_INVALID_ARG, "null argument");
    *stream = (void*)ctx->stream;
    return OCEAN_OK;
}

int ocean_synchronize(ocean_ctx* ctx) {
    OCEAN_ENTER(ctx);
    OCEAN_HIP(hipStreamSynchronize(ctx->stream));
    return OCEAN_OK;
}

// (the caller has entered: OCEAN_ENTER)
static int check_sample(ocean_ctx* ctx, int tile, const float* pts, int count, float* out) {
    if (tile < 0 || tile >= ctx->T) return fail(OCEAN_E_INVALID_ARG, "tile out of range");
    if (count < 0) return fail(OCEAN_E_INVALID_ARG, "negative point count");
    if (count > 0 && (!pts || !out)) return fail(OCEAN_E_INVALID_ARG, "null points or output");
    // the cascade constants (wavelengths) the sampler divides by exist only after init
    if (!ctx->spectrum_ready) return fail(OCEAN_E_STATE, "ocean_init_spectrum must precede ocean_sample_world");
    return OCEAN_OK;
}

int ocean_sample_world_device(ocean_ctx* ctx, int tile, const float* points, int count, float* out) {
    OCEAN_ENTER(ctx);
    if (int r = check_sample(ctx, tile, points, count, out)) return r;
    if (ctx->col_par >= 0) return fail(OCEAN_E_UNSUPPORTED, "world sampling of a column-parity shard (half the columns)");
    // k_sample_world reads floats and writes float4 rows (ocean.h)
    if (((uintptr_t)points & 3) || ((uintptr_t)out & 15))
        return fail(OCEAN_E_INVALID_ARG, "ocean_sample_world_device: points must be 4-byte and out 16-byte aligned");
    const ocean::DevView v = ctx->view();
    return timed(ctx, 2, [&] { return ocean::launch_sample_world(v, tile, points, count, out, ctx->stream); },
                 "sample_world");
}

int ocean_sample_world(ocean_ctx* ctx, int tile, const float* points, int count, float* out) {
    OCEAN_ENTER(ctx);
    if (int r = check_sample(ctx, tile, points, count, out)) return r;
    if (count == 0) return OCEAN_OK;
    const size_t in_bytes = (size_t)count * 3 * 4, out_bytes = (size_t)count * 12 * 4;
    const size_t out_off = (in_bytes + 255) & ~(size_t)255;  // float4 output rows stay 16-B aligned
    void* d = nullptr;
    OCEAN_HIP(hipMallocAsync(&d, out_off + out_bytes, ctx->stream));
    float* d_in = static_cast<float*>(d);
    float* d_out = reinterpret_cast<float*>(static_cast<char*>(d) + out_off);
    hipError_t e = hipMemcpyAsync(d_in, points, in_bytes, hipMemcpyHostToDevice, ctx->stream);
    int r = OCEAN_OK;
    if (e == hipSuccess) r = ocean_sample_world_device(ctx, tile, d_in, count, d_out);
    if (e == hipSuccess && r == OCEAN_OK) e = hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream);
    const hipError_t ef = hipFreeAsync(d, ctx->stream);
    const hipError_t es = hipStreamSynchronize(ctx->stream);
    if (r != OCEAN_OK) return r;
    if (e != hipSuccess) return hip_fail(e, "ocean_sample_world copy");
    if (ef != hipSuccess) return hip_fail(ef, "hipFreeAsync");
    if (es != hipSuccess) return hip_fail(es, "hipStreamSynchronize");
    return OCEAN_OK;
}

int ocean_set_column_band(ocean_ctx* ctx, int x_begin, int x_count) {
    OCEAN_ENTER(ctx);
    const int n = ctx->n;
    const int g = std::min(n, std::max(16, 8192 / n));  // a multiple of every tile width of the fused passes
    if (x_begin < 0 || x_count < 1 || x_begin + x_count > n || x_begin % g || x_count % g)
        return fail(OCEAN_E_INVALID_ARG, "column band [" + std::to_string(x_begin) + ", +" + std::to_string(x_count) +
                                             ") must lie in [0, N) with start and width multiples of " +
                                             std::to_string(g));
    if (x_count != n && (ctx->flags & (OCEAN_F_UNFUSED | OCEAN_F_MIPS)))
        return fail(OCEAN_E_UNSUPPORTED, "a column band needs the fused schedule and no mip chains");
    ctx->band_x0 = x_begin;
    ctx->band_nx = x_count;
    ctx->col_par = -1;  // a band replaces a column parity
    return OCEAN_OK;
}

int ocean_set_column_parity(ocean_ctx* ctx, int parity) {
    OCEAN_ENTER(ctx);
    if (parity < -1 || parity > 1) return fail(OCEAN_E_INVALID_ARG, "parity must be -1 (off), 0 or 1");
    if (parity < 0) {
        ctx->col_par = -1;
        ctx->band_x0 = 0;
        ctx->band_nx = ctx->n;
        return OCEAN_OK;
    }
    if (ctx->n != 4096) return fail(OCEAN_E_UNSUPPORTED, "a column parity is built for N = 4096 (pass A3P)");
    if (ctx->flags & (OCEAN_F_UNFUSED | OCEAN_F_MIPS | OCEAN_F_DISPLACEMENT_ONLY))
        return fail(OCEAN_E_UNSUPPORTED, "a column parity needs the fused full-output schedule and no mip chains");
    if (!ctx->opt.q) return fail(OCEAN_E_UNSUPPORTED, "a column parity needs the three-plane frame (OCEAN_Q=0 is set)");
    // pass A3PP reads h0(k) of mirror-pair rows from h0k (8 B per texel instead of h0's 16): allocated on
    // the first parity, then kept up to date by ocean_init_spectrum (k_conjugate writes it)
    if (!ctx->h0k) {
        const size_t bytes = ctx->texels() * ctx->units() * 8;
        OCEAN_HIP(hipMalloc((void**)&ctx->h0k, bytes));
        ctx->h0k_valid = false;
    }
    // extract whenever the spectrum exists (h0.zw = conj h0(-k)) and h0k does not match it yet: a failed
    // extract leaves h0k_valid false, so the next call retries it; before ocean_init_spectrum there is
    // nothing to extract, and the init fills h0k itself
    if (!ctx->h0k_valid && ctx->h0_conj) {
        const ocean::DevView v = ctx->view();
        OCEAN_HIP(ocean::launch_h0k_extract(v, ctx->stream));
        OCEAN_HIP(hipStreamSynchronize(ctx->stream));
        ctx->h0k_valid = true;
    }
    ctx->col_par = parity;
    ctx->band_x0 = 0;
    ctx->band_nx = ctx->n / 2;  // compact: column m of every texture holds x = 2 m + parity
    return OCEAN_OK;
}

int ocean_set_kernel_timing(ocean_ctx* ctx, int enable) {
    OCEAN_ENTER(ctx);
    if (enable && ctx->event_pool.size() < 4096) {
        // pre-create events so the timed region never creates any
        while (ctx->event_pool.size() < 4096) {
            hipEvent_t e = nullptr;
            OCEAN_HIP(hipEventCreate(&e));
            ctx->event_pool.push_back(e);
        }
    }
    if (!enable && !ctx->pending.empty())  // launches timed so far still count at the next ocean_kernel_stats
        if (int r = fold_pending(ctx, true)) return r;
    ctx->timing = enable != 0;
    return OCEAN_OK;
}

int ocean_step_bytes(ocean_ctx* ctx, uint64_t* pass_a, uint64_t* pass_b) {
    if (!ctx || !pass_a || !pass_b) return fail(OCEAN_E_INVALID_ARG, "null argument");
    const uint64_t tex = (uint64_t)ctx->texels() * ctx->units();
    const uint64_t P = ctx->P;
    const bool full = P == 4, normals = (ctx->flags & OCEAN_F_NORMALS) != 0;
    const uint64_t outs = 16 + (full ? 32 : 0) + (normals ? 16 : 0);  // DISP [+ DERIV + TURB] [+ NORMAL]
    uint64_t a = 0, b = 0;
    if (ctx->flags & OCEAN_F_UNFUSED) {
        // evolve: h0 + waves -> P planes; rows and columns: read + write every plane;
        // fill: P planes [+ foam state read + write] -> outputs
        a = tex * (32 + 8 * P + 16 * P);
        b = tex * (16 * P + 8 * P + (full ? 8 : 0) + outs);
    } else {
        const bool a4 = ctx->opt.a4 && ctx->h0k_valid && ocean::pass_a4_supported(ctx->n, ctx->P);
        // column band: h0 is read whole (rows are transformed whole), the rest scales with the band
        const uint64_t bt = tex / ctx->n * ctx->band_nx;
        if (use_q(ctx)) {
            // three-plane frame (the side arrays, 16 B per row, not counted): pass A h0k (h0 at
            // N >= 2048) -> Q1..Q3; pass B Q1..Q3 + foam state -> outputs, or at N >= 2048 the
            // four-step passes: C1 reads Q1..Q3 and writes them with R[Q4], C2 reads four planes
            // the column-parity row pass on mirror-pair rows (pass A3PP) reads h0k, 8 B per texel
            const bool h0k_pairs = ctx->col_par >= 0;
            *pass_a = tex * ((ctx->n >= 2048 && !h0k_pairs) ? 16 : 8) + bt * 24;
            *pass_b = ctx->n >= 2048 ? bt * (24 + 32 + 32 + 8 + outs) : bt * (24 + 8 + outs);
            return OCEAN_OK;
        }
        a = tex * (a4 ? 8 : 16) + bt * 8 * P;
        b = bt * (8 * P + (full ? 8 : 0) + outs);  // + foam state read and write
        if (ocean::pass_c4_supported(ctx->n)) b += bt * 16 * P;  // four-step: step 1 reads + writes the planes
    }
    *pass_a = a;
    *pass_b = b;
    return OCEAN_OK;
}

int ocean_kernel_name(ocean_ctx* ctx, int kind, char* buf, size_t len) {
    if (!ctx || !buf || len == 0) return fail(OCEAN_E_INVALID_ARG, "null argument or zero length");
    if (kind < 0 || kind > 2) return fail(OCEAN_E_INVALID_ARG, "bad kind");
    buf[0] = 0;
    if (!ctx->kind_kernel[kind]) return fail(OCEAN_E_STATE, "no kernel of this kind launched yet");
    OCEAN_ENTER(ctx);
    const char* mangled = hipKernelNameRefByPtr(ctx->kind_kernel[kind], ctx->stream);
    if (!mangled) return fail(OCEAN_E_DEVICE, "hipKernelNameRefByPtr returned no name");
    int st = 0;
    char* dem = abi::__cxa_demangle(mangled, nullptr, nullptr, &st);
    const std::string name = (st == 0 && dem) ? dem : mangled;
    std::free(dem);
    std::snprintf(buf, len, "%s", name.c_str());
    return name.size() < len ? OCEAN_OK : fail(OCEAN_E_INVALID_ARG, "buffer too small for " + name);
}

int ocean_kernel_stats(ocean_ctx* ctx, int kind, double* total_ms, long long* launches) {
    OCEAN_ENTER(ctx);
    if (kind < 0 || kind > 2 || !total_ms || !launches) return fail(OCEAN_E_INVALID_ARG, "bad kind or null output");
    if (int r = fold_pending(ctx, true)) return r;
    *total_ms = ctx->kind_ms[kind];
    *launches = ctx->kind_count[kind];
    ctx->kind_ms[kind] = 0;
    ctx->kind_count[kind] = 0;
    return OCEAN_OK;
}

}  // extern "C"
