// abi_host: a compiled, non-Python host walking the reference's WaterBody lifecycle
// through the C ABI (water_body.h): Awake -> Update x F (a readback request every
// frame) -> GetWaterHeight -> OnValidate (re-init, foam kept) -> Update -> SampleWorld
// -> OnDisable.  tests/test_gpu_host.py runs it and checks every number it writes
// against the same sequence through the Python binding and against the oracle.
//
//   abi_host <outdir> <n> <cascades> <frames> [height|rgba]
//
// The readback mode (water_body.h Readback) defaults to height.  Writes <outdir>/buoyancy0.bin
// (buoyancyData after the first F frames, float32 [n][n] heights, or [n][n][4] with rgba),
// buoyancy1.bin (after OnValidate + one frame), heights.bin (float32
// [F][4]: GetWaterHeight at 4 world points after each Update), sample.bin (float32
// [8][12], SampleWorld of 8 points) and prints one JSON summary line.
#include <cstdio>
#include <cstdlib>
#include <string>

#include "water_body.h"

namespace {

void write_bin(const std::string& path, const float* data, size_t count) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f || std::fwrite(data, sizeof(float), count, f) != count) {
        std::fprintf(stderr, "cannot write %s\n", path.c_str());
        std::exit(2);
    }
    std::fclose(f);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 5 && argc != 6) {
        std::fprintf(stderr, "usage: %s <outdir> <n> <cascades> <frames> [height|rgba]\n", argv[0]);
        return 2;
    }
    const std::string mode = argc == 6 ? argv[5] : "height";
    if (mode != "height" && mode != "rgba") {
        std::fprintf(stderr, "usage: readback mode must be height or rgba\n");
        return 2;
    }
    const std::string out = argv[1];
    const int n = std::atoi(argv[2]), C = std::atoi(argv[3]), F = std::atoi(argv[4]);
    // the reference scene (Assets/Scenes/Waves.unity:1305-1322; cascades :1431-1435,
    // :470-474, :1249-1253 and the unreferenced 4th :1572-1576)
    const ocean_host::WaterCascade scene[4] = {
        {1530.0f, 1e12f, 1e-10f, 0.4f, 0.1f}, {1000.0f, 1e7f, 1e-7f, 0.3f, 0.2f},
        {201.0f, 1e6f, 1e-5f, 0.1f, 0.1f}, {34.0f, 10.0f, 0.001f, 0.4f, 0.1f}};
    try {
        ocean_host::WaterBody wb;
        wb.windSpeed = 8.0f;
        wb.windDirectionX = 1.0f;
        wb.windDirectionY = -1.0f;
        wb.gravity = 9.81f;
        wb.fetch = 50000.0f;
        wb.depth = 2560.0f;
        wb.texturesSize = n;
        wb.cascades.assign(scene, scene + (C < 4 ? C : 4));
        wb.seed = 42;
        wb.readback = mode == "height" ? ocean_host::Readback::Height : ocean_host::Readback::Rgba;
        wb.Awake();
        const float probe[4][2] = {{0.0f, 0.0f}, {-(float)n / 2, -(float)n / 2}, {(float)n / 2 - 1, 50.0f}, {500.0f, -500.0f}};
        std::vector<float> heights;
        for (int f = 0; f < F; ++f) {
            wb.Update((float)f / 60.0f);
            for (auto& p : probe) heights.push_back(wb.GetWaterHeight(p[0], p[1]));
        }
        wb.WaitForReadbacks();
        {
            const std::vector<float>& buoy = wb.buoyancyData();
            write_bin(out + "/buoyancy0.bin", buoy.data(), buoy.size());
        }
        write_bin(out + "/heights.bin", heights.data(), heights.size());
        wb.windSpeed = 12.0f;
        wb.OnValidate();
        wb.Update(0.5f);
        wb.WaitForReadbacks();
        {
            const std::vector<float>& buoy = wb.buoyancyData();
            write_bin(out + "/buoyancy1.bin", buoy.data(), buoy.size());
        }
        std::vector<float> pts;
        for (int i = 0; i < 8; ++i) {
            pts.push_back(-300.0f + 97.5f * i);
            pts.push_back(40.0f - 13.25f * i);
            pts.push_back(0.5f * i);
        }
        const std::vector<float> s = wb.SampleWorld(pts);
        write_bin(out + "/sample.bin", s.data(), s.size());
        std::printf("{\"frames\": %d, \"requested\": %ld, \"completed\": %ld, \"n\": %d, \"cascades\": %d}\n", F + 1,
                    wb.requested(), wb.completed(), n, (int)wb.cascades.size());
        wb.OnDisable();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "abi_host: %s\n", e.what());
        return 1;
    }
    return 0;
}
