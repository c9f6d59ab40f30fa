// WaterBody-shaped C++ host over the C ABI (include/ocean/ocean.h): the lifecycle of
// Assets/Scripts/Water/WaterBody.cs -- Awake (:211-256), the commented OnValidate
// re-init (:324-337), Update with an AsyncGPUReadback request EVERY frame (:284-297),
// GetWaterHeight (:195-209), OnDisable (:300-309) -- written the way a non-Python host
// binds the library.  It mirrors csharp/WaterBodyNative.cs call for call (the C# host
// cannot be compiled in this image: no dotnet), and abi_host.cpp drives it in a -m gpu
// test.  Header-only; errors throw std::runtime_error with ocean_last_error().
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <string>
#include <vector>

#include "ocean/ocean.h"

namespace ocean_host {

inline void check(int rc, const char* where) {
    if (rc != OCEAN_OK) throw std::runtime_error(std::string(where) + " failed (" + std::to_string(rc) + "): " +
                                                 ocean_last_error());
}

// What Update reads back every frame: the height channel GetWaterHeight reads (ocean_read_height_async,
// 4 B per texel; the reference's buoyancyData is private, WaterBody.cs:58, and .g is all its reader uses)
// or the whole RGBA displacement slice (ocean_read_async, 16 B per texel) as the reference requests it.
enum class Readback { Height, Rgba };

struct WaterCascade {  // WaterCascade.cs:10-24 (script defaults)
    float wavelength = 10.0f, cutoffHigh = 5.0f, cutoffLow = 0.0001f, swell = 0.4f, fade = 0.1f;
};

class WaterBody {
public:
    // WaterBody.cs:10-14, :29 (script defaults)
    float windSpeed = 1.0f, windDirectionX = 1.0f, windDirectionY = 1.0f;
    float gravity = 9.81f, fetch = 1.0f, depth = 4.0f;
    int texturesSize = 256;
    std::vector<WaterCascade> cascades{WaterCascade{}};
    uint64_t seed = 20251121;  // the reference's UnityEngine.Random is unseeded; this library's generator is
    int device = 0;
    size_t maxReadbacksInFlight = 4;  // bound on queued requests (set before Awake): 2-4 keep the copies back to
                                      // back beside the frames; 8 stretch each
    Readback readback = Readback::Height;  // set before Awake

    WaterBody() = default;
    WaterBody(const WaterBody&) = delete;
    WaterBody& operator=(const WaterBody&) = delete;
    ~WaterBody() { OnDisable(); }

    void Awake() {
        check(ocean_create(device, texturesSize, (int)cascades.size(), 1, OCEAN_F_MIPS, &ctx_), "ocean_create");
        ApplyParams();
        check(ocean_generate_noise(ctx_, seed), "ocean_generate_noise");
        check(ocean_init_spectrum(ctx_), "ocean_init_spectrum");
        // the readback ring: maxReadbacksInFlight pinned slices, plus the one the last landed slice stays
        // in, allocated once and reused, freed only in OnDisable (hipHostFree synchronizes the device,
        // so a free per request would make every Update wait for the frame it just queued)
        for (size_t i = 0; i < std::max<size_t>(maxReadbacksInFlight, 1) + 1; ++i) {
            void* b = nullptr;
            check(ocean_host_alloc(SliceBytes(), &b), "ocean_host_alloc");
            free_.push_back(b);
            owned_.push_back(b);
        }
    }

    // Parameter change -> spectrum re-init; the foam accumulator carries over, as there.
    void OnValidate() {
        if (!ctx_) return;
        ApplyParams();
        check(ocean_init_spectrum(ctx_), "ocean_init_spectrum");
    }

    void CalculateWavesTexturesAtTime(float time) { check(ocean_step(ctx_, time), "ocean_step"); }

    // Step, then request the displacement slice 0; requests complete in order and each
    // completed one refreshes buoyancyData (the reference's callback, :292-295).
    void Update(float time) {
        CalculateWavesTexturesAtTime(time);
        while (!readbacks_.empty()) {
            const int st = ocean_readback_status(readbacks_.front().req);
            if (st == 0) break;
            Complete(st);
        }
        // at most maxReadbacksInFlight requests queued (the ring's extra slot holds the landed slice):
        // when full, wait for the oldest
        while (!readbacks_.empty() && (readbacks_.size() >= std::max<size_t>(maxReadbacksInFlight, 1) || free_.empty())) {
            const int st = ocean_readback_wait(readbacks_.front().req) == OCEAN_OK ? 1 : -1;
            Complete(st);
        }
        Pending p;
        p.buf = free_.back();
        free_.pop_back();
        const int rc = readback == Readback::Height
                           ? ocean_read_height_async(ctx_, 0, 0, static_cast<float*>(p.buf), SliceBytes(), &p.req)
                           : ocean_read_async(ctx_, OCEAN_TEX_DISP, 0, 0, p.buf, SliceBytes(), &p.req);
        if (rc != OCEAN_OK) {
            free_.push_back(p.buf);
            check(rc, readback == Readback::Height ? "ocean_read_height_async" : "ocean_read_async");
        }
        readbacks_.push_back(p);
        ++requested_;
    }

    void WaitForReadbacks() {
        while (!readbacks_.empty()) {
            const int st = ocean_readback_wait(readbacks_.front().req) == OCEAN_OK ? 1 : -1;
            Complete(st);
        }
    }

    // WaterBody.cs:195-209, with its mapping of world x, z over [-texturesSize/2, texturesSize/2].
    float GetWaterHeight(float worldX, float worldZ) const {
        if (!held_) return 0.0f;
        auto inverse_lerp = [](float a, float b, float v) {
            return a == b ? 0.0f : std::min(std::max((v - a) / (b - a), 0.0f), 1.0f);
        };
        const int n = texturesSize;
        const float u = inverse_lerp((float)(-n / 2), (float)(n / 2), worldX);
        const float v = inverse_lerp((float)(-n / 2), (float)(n / 2), worldZ);
        const int x = std::min(std::max((int)(u * n), 0), n - 1);
        const int y = std::min(std::max((int)(v * n), 0), n - 1);
        const size_t t = (size_t)y * n + x;
        return readback == Readback::Height ? held_[t] : held_[t * 4 + 1];  // .g = Dy
    }

    // What Water.shader reads at world positions (x, z, lod) -> 12 floats per point.
    std::vector<float> SampleWorld(const std::vector<float>& points) const {
        std::vector<float> out(points.size() / 3 * 12);
        check(ocean_sample_world(ctx_, 0, points.data(), (int)(points.size() / 3), out.data()), "ocean_sample_world");
        return out;
    }

    std::vector<float> ReadSlice(int texture, int cascade) const {
        std::vector<float> out(SliceBytes() / 4);
        check(ocean_read(ctx_, texture, 0, cascade, out.data(), SliceBytes()), "ocean_read");
        return out;
    }

    void OnDisable() {
        for (auto& p : readbacks_) ocean_readback_release(p.req);
        readbacks_.clear();
        if (held_slot_) {  // the last landed slice outlives the pinned ring
            last_.assign(held_, held_ + SliceBytes() / 4);
            held_ = last_.data();
            held_slot_ = nullptr;
        }
        for (void* b : owned_) ocean_host_free(b);
        owned_.clear();
        free_.clear();
        if (ctx_) ocean_destroy(ctx_);
        ctx_ = nullptr;
    }

    // The last landed displacement slice 0 (WaterBody.cs:295's array): [y][x] heights (Readback::Height)
    // or [y][x][rgba] (Readback::Rgba); empty before the first readback lands.  Copied out of its pinned slot once, on the first call after it lands; later
    // calls return the same array until the next readback lands (the reference reads a field).
    const std::vector<float>& buoyancyData() {
        if (held_ && !buoy_valid_) {
            buoy_.assign(held_, held_ + SliceBytes() / 4);
            buoy_valid_ = true;
        }
        if (!held_) buoy_.clear();
        return buoy_;
    }
    long requested() const { return requested_; }
    long completed() const { return completed_; }

private:
    struct Pending {
        ocean_readback* req = nullptr;
        void* buf = nullptr;
    };
    ocean_ctx* ctx_ = nullptr;
    std::deque<Pending> readbacks_;
    std::vector<void*> free_, owned_;  // pinned readback ring: idle slots, all slots
    const float* held_ = nullptr;  // the last landed slice, in its pinned slot (out of the ring)
    void* held_slot_ = nullptr;
    std::vector<float> last_;  // the last slice after OnDisable
    std::vector<float> buoy_;  // buoyancyData's copy of the held slice
    bool buoy_valid_ = false;
    long requested_ = 0, completed_ = 0;

    size_t SliceBytes() const { return (size_t)texturesSize * texturesSize * (readback == Readback::Height ? 4 : 16); }

    void ApplyParams() {
        ocean_params p{windSpeed, windDirectionX, windDirectionY, gravity, fetch, depth};
        std::vector<ocean_cascade> cs;
        for (const auto& c : cascades) cs.push_back({c.wavelength, c.cutoffLow, c.cutoffHigh, c.swell, c.fade});
        check(ocean_set_params(ctx_, &p, cs.data()), "ocean_set_params");
    }

    // st: 1 done, < 0 request.hasError (data dropped, as the reference's callback does)
    void Complete(int st) {
        Pending p = readbacks_.front();
        readbacks_.pop_front();
        ocean_readback_release(p.req);
        if (st == 1) {
            // The reference copies every landed request out (request.GetData<Color>().ToArray(),
            // :295): Unity's NativeArray lives only inside the callback.  The pinned slot outlives
            // the request, so the slice stays in place and the slot leaves the ring until the next
            // landed readback replaces it (no 16 MiB host copy per frame at 1024^2).
            if (held_slot_) free_.push_back(held_slot_);
            held_slot_ = p.buf;
            held_ = static_cast<const float*>(p.buf);
            buoy_valid_ = false;
            ++completed_;
        } else {
            free_.push_back(p.buf);  // back to the ring
        }
    }
};

}  // namespace ocean_host
