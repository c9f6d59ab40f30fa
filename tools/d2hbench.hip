// Device-to-host readback on MI355X: which engine carries a 16 MiB
// hipMemcpyAsync into pinned host memory, its own bandwidth, and what it does to a concurrent
// frame.  The frame stand-in is a streaming kernel over 256 MiB (read + write, every CU busy for
// about the time of a cfg3 frame); the copy runs on a second stream, as ocean_read_async's does.
//   kinds: D2H (hipMemcpyDeviceToHost), DEF (hipMemcpyDefault), NOCU (hipMemcpyDeviceToDeviceNoCU:
//   the runtime's "no compute units" copy, i.e. an SDMA engine), per host allocation flag.
// Prints the GPU's NUMA node and the calling CPU's, since a pinned buffer on the far socket halves
// the link rate.
// Build: hipcc --offload-arch=gfx950 -O3 tools/d2hbench.hip -o tools/d2hbench
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_frame(const f32x4* __restrict__ in, f32x4* __restrict__ out, size_t n4, float s) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        f32x4 v = in[i];
        v.x += s;
        __builtin_nontemporal_store(v, out + i);
    }
}

static int read_int_file(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return -2;
    int v = -2;
    if (std::fscanf(f, "%d", &v) != 1) v = -2;
    std::fclose(f);
    return v;
}

// NUMA node of the page holding addr (get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR)), -1 if unknown
static int page_node(const void* addr) {
    int node = -1;
    const long r = syscall(SYS_get_mempolicy, &node, nullptr, 0UL, addr, 3UL /* MPOL_F_NODE | MPOL_F_ADDR */);
    return r == 0 ? node : -1;
}

// Restrict the calling thread to the CPUs of `node` that it may already run on; false if none.
static bool bind_to_node(int node) {
    cpu_set_t cur, want;
    if (sched_getaffinity(0, sizeof(cur), &cur) != 0) return false;
    CPU_ZERO(&want);
    FILE* f = std::fopen(("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str(), "r");
    if (!f) return false;
    char buf[4096] = {0};
    const size_t got = std::fread(buf, 1, sizeof(buf) - 1, f);
    std::fclose(f);
    buf[got] = 0;
    int count = 0;
    for (char* tok = std::strtok(buf, ",\n"); tok; tok = std::strtok(nullptr, ",\n")) {
        int a = 0, b = 0;
        if (std::sscanf(tok, "%d-%d", &a, &b) == 2) {
        } else if (std::sscanf(tok, "%d", &a) == 1) {
            b = a;
        } else {
            continue;
        }
        for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(c, &cur)) {
                CPU_SET(c, &want);
                ++count;
            }
    }
    return count > 0 && sched_setaffinity(0, sizeof(want), &want) == 0;
}

static int cpu_node(int cpu) {
    for (int node = 0; node < 16; ++node) {
        std::string p = "/sys/devices/system/node/node" + std::to_string(node) + "/cpu" + std::to_string(cpu);
        FILE* f = std::fopen((p + "/online").c_str(), "r");
        if (f) {
            std::fclose(f);
            return node;
        }
        // cpu0 has no "online" file: test the directory through its topology entry
        f = std::fopen((p + "/topology/core_id").c_str(), "r");
        if (f) {
            std::fclose(f);
            return node;
        }
    }
    return -1;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
    const size_t slice = 16u << 20;  // one 1024^2 float4 slice (DISP slice 0)
    const size_t big = 256u << 20;   // the frame stand-in's bytes, each direction
    char bus[64] = {0};
    CK(hipDeviceGetPCIBusId(bus, sizeof(bus), 0));
    for (char* p = bus; *p; ++p) *p = (char)std::tolower(*p);
    const int gpu_node = read_int_file(std::string("/sys/bus/pci/devices/") + bus + "/numa_node");
    const int cpu = sched_getcpu();
    printf("gpu pci %s numa_node %d; calling cpu %d numa_node %d\n", bus, gpu_node, cpu, cpu_node(cpu));

    void *src = nullptr, *fin = nullptr, *fout = nullptr;
    CK(hipMalloc(&src, slice));
    CK(hipMalloc(&fin, big));
    CK(hipMalloc(&fout, big));
    CK(hipMemset(src, 1, slice));
    CK(hipMemset(fin, 0, big));
    hipStream_t s_frame, s_copy;
    CK(hipStreamCreateWithFlags(&s_frame, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s_copy, hipStreamNonBlocking));
    hipEvent_t a, b, c, d;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreate(&c));
    CK(hipEventCreate(&d));
    const int grid = 256 * 8, block = 256;
    const size_t n4 = big / 16;
    const int frame_kernels = 4;  // ~ the frame's two passes x 2

    auto frame = [&]() -> hipError_t {
        for (int k = 0; k < frame_kernels; ++k) {
            k_frame<<<grid, block, 0, s_frame>>>((const f32x4*)fin, (f32x4*)fout, n4, 1.0f);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    };
    // frame alone
    for (int w = 0; w < 10; ++w) CK(frame());
    CK(hipStreamSynchronize(s_frame));
    CK(hipEventRecord(a, s_frame));
    for (int r = 0; r < reps; ++r) CK(frame());
    CK(hipEventRecord(b, s_frame));
    CK(hipEventSynchronize(b));
    float ms_frame = 0;
    CK(hipEventElapsedTime(&ms_frame, a, b));
    printf("frame alone                 %9.1f us per frame (%d kernels over %zu MiB)\n", 1e3 * ms_frame / reps,
           frame_kernels, big >> 20);

    struct HostKind {
        const char* name;
        unsigned flags;
    } hosts[] = {{"default", hipHostMallocDefault},
                 {"numa_user", hipHostMallocNumaUser},
                 {"noncoherent", hipHostMallocNonCoherent},
                 {"coherent", hipHostMallocCoherent}};
    struct CopyKind {
        const char* name;
        hipMemcpyKind kind;
    } kinds[] = {{"D2H", hipMemcpyDeviceToHost}, {"DEF", hipMemcpyDefault}, {"NOCU", hipMemcpyDeviceToDeviceNoCU}};

  // d2hbench reps [host kind index [ring kind name]]: one host kind's ring runs only (rocprofv3 runs)
  const int only = argc > 2 ? std::atoi(argv[2]) : -1;
  for (int phase = 0; phase < 3; ++phase) {
    if (phase > 0 && only >= 0) break;
    if (phase == 1) {
        // memory policy of the calling thread: prefer the GPU's node, with hipHostMallocNumaUser
        unsigned long mask = 1UL << (gpu_node < 0 ? 0 : gpu_node);
        const long r = syscall(SYS_set_mempolicy, 1 /* MPOL_PREFERRED */, &mask, 64UL);
        printf("-- set_mempolicy(MPOL_PREFERRED, node %d): %s\n", gpu_node, r == 0 ? "ok" : "failed");
        if (r != 0) break;
    }
    if (phase == 2) {
        if (gpu_node < 0 || !bind_to_node(gpu_node)) {
            printf("cannot bind to the GPU's NUMA node %d\n", gpu_node);
            break;
        }
        const int c2 = sched_getcpu();
        printf("-- thread bound to the GPU's node: cpu %d numa_node %d\n", c2, cpu_node(c2));
    }
    for (const HostKind& h : hosts) {
        if (only >= 0 && &h - hosts != only) continue;
        void* dst = nullptr;
        if (hipHostMalloc(&dst, slice, h.flags) != hipSuccess) {
            printf("host %-12s hipHostMalloc failed\n", h.name);
            (void)hipGetLastError();
            continue;
        }
        std::memset(dst, 0, slice);
        printf("host %-12s pages on numa_node %d\n", h.name, page_node(dst));
        for (const CopyKind& k : kinds) {
            if (only >= 0) break;
            // copy alone
            hipError_t e = hipMemcpyAsync(dst, src, slice, k.kind, s_copy);
            if (e != hipSuccess) {
                printf("host %-12s %-5s hipMemcpyAsync: %s\n", h.name, k.name, hipGetErrorString(e));
                (void)hipGetLastError();
                continue;
            }
            CK(hipStreamSynchronize(s_copy));
            CK(hipEventRecord(c, s_copy));
            for (int r = 0; r < reps; ++r) CK(hipMemcpyAsync(dst, src, slice, k.kind, s_copy));
            CK(hipEventRecord(d, s_copy));
            CK(hipEventSynchronize(d));
            float ms_copy = 0;
            CK(hipEventElapsedTime(&ms_copy, c, d));
            const double us_copy = 1e3 * ms_copy / reps;
            // copy beside the frame: one copy per frame, both streams busy
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a, s_frame));
            CK(hipEventRecord(c, s_copy));
            for (int r = 0; r < reps; ++r) {
                CK(frame());
                CK(hipMemcpyAsync(dst, src, slice, k.kind, s_copy));
            }
            CK(hipEventRecord(b, s_frame));
            CK(hipEventRecord(d, s_copy));
            CK(hipEventSynchronize(b));
            CK(hipEventSynchronize(d));
            float mf = 0, mc = 0;
            CK(hipEventElapsedTime(&mf, a, b));
            CK(hipEventElapsedTime(&mc, c, d));
            // check the bytes landed
            const unsigned char* p = (const unsigned char*)dst;
            const bool ok = p[0] == 1 && p[slice - 1] == 1;
            printf("host %-12s %-5s alone %8.1f us %6.1f GB/s | beside frame: frame %8.1f us (x%.2f), copy %8.1f us "
                   "%6.1f GB/s%s\n",
                   h.name, k.name, us_copy, slice / us_copy / 1e3, 1e3 * mf / reps, mf / ms_frame,
                   1e3 * mc / reps, slice / (1e3 * mc / reps) / 1e3, ok ? "" : "  DATA MISMATCH");
            std::memset(dst, 0, slice);
        }
        for (const CopyKind& k : kinds) {
            if (k.kind == hipMemcpyDefault) continue;
            if (argc > 3 && std::strcmp(argv[3], k.name) != 0) continue;  // one ring kind (rocprofv3 runs)
            // ocean_read_async's sequence per frame: the snapshot (device copy into a staging slot) on
            // the frame stream, an event, the copy stream waits for it, then the device-to-host copy
            void* stage = nullptr;
            CK(hipMalloc(&stage, slice));
            hipEvent_t after;
            CK(hipEventCreateWithFlags(&after, hipEventDisableTiming));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a, s_frame));
            CK(hipEventRecord(c, s_copy));
            for (int r = 0; r < reps; ++r) {
                CK(frame());
                CK(hipMemcpyAsync(stage, src, slice, hipMemcpyDeviceToDevice, s_frame));
                CK(hipEventRecord(after, s_frame));
                CK(hipStreamWaitEvent(s_copy, after, 0));
                CK(hipMemcpyAsync(dst, stage, slice, k.kind, s_copy));
            }
            CK(hipEventRecord(b, s_frame));
            CK(hipEventRecord(d, s_copy));
            CK(hipEventSynchronize(b));
            CK(hipEventSynchronize(d));
            float mf = 0, mc = 0;
            CK(hipEventElapsedTime(&mf, a, b));
            CK(hipEventElapsedTime(&mc, c, d));
            const unsigned char* p = (const unsigned char*)dst;
            printf("host %-12s ring %-4s snapshot + wait + copy per frame: frame stream %8.1f us (x%.2f), copy stream %8.1f us "
                   "per frame%s\n", h.name, k.name, 1e3 * mf / reps, mf / ms_frame, 1e3 * mc / reps,
                   (p[0] == 1 && p[slice - 1] == 1) ? "" : "  DATA MISMATCH");
            CK(hipEventDestroy(after));
            CK(hipFree(stage));
        }
        CK(hipHostFree(dst));
    }
  }
    return 0;
}
