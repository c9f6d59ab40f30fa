// Host-side Gaussian noise texture, the reference's GenerateRandomNoiseTexture
// (WaterBody.cs:86-100) with GenerateRandomNumber (WaterBody.cs:71-81):
// Marsaglia polar method, keep v1 * s, texel (x = i, y = j) = (g1, g2),
// generated with i (x) outer and j (y) inner.  The reference draws its
// uniforms from UnityEngine.Random (closed source, never seeded); this library
// documents its own source: xorshift128 (Marsaglia 2003) whose 128-bit state is
// filled by two splitmix64 outputs of `seed`, U = (u32 >> 8) * 2^-24.
// Init-only, as in the reference (it runs once in Awake on the CPU).
#include <cmath>
#include <cstddef>
#include <cstdint>

namespace ocean {
namespace {

struct Xorshift128 {
    uint32_t s[4];

    static uint64_t splitmix64(uint64_t& x) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }

    explicit Xorshift128(uint64_t seed) {
        uint64_t x = seed;
        const uint64_t a = splitmix64(x), b = splitmix64(x);
        s[0] = (uint32_t)a;
        s[1] = (uint32_t)(a >> 32);
        s[2] = (uint32_t)b;
        s[3] = (uint32_t)(b >> 32);
        if ((s[0] | s[1] | s[2] | s[3]) == 0) s[0] = 1u;
    }

    uint32_t next() {
        const uint32_t t = s[0] ^ (s[0] << 11);
        s[0] = s[1];
        s[1] = s[2];
        s[2] = s[3];
        s[3] = s[3] ^ (s[3] >> 19) ^ t ^ (t >> 8);
        return s[3];
    }

    float uniform() { return (float)(next() >> 8) * (1.0f / 16777216.0f); }

    float gaussian() {  // WaterBody.cs:71-81
        float v1, v2, q;
        do {
            v1 = 2.0f * uniform() - 1.0f;
            v2 = 2.0f * uniform() - 1.0f;
            q = v1 * v1 + v2 * v2;
        } while (q >= 1.0f || q == 0.0f);
        q = std::sqrt((-2.0f * std::log(q)) / q);
        return v1 * q;
    }
};

}  // namespace

// out: float2[N][N] laid out [y][x].
void generate_noise_host(int n, uint64_t seed, float* out) {
    Xorshift128 rng(seed);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            const float g1 = rng.gaussian();
            const float g2 = rng.gaussian();
            out[((size_t)j * n + i) * 2 + 0] = g1;
            out[((size_t)j * n + i) * 2 + 1] = g2;
        }
}

}  // namespace ocean
