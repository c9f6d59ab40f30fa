// The C# CPU baseline harness of SURVEY.md 8d: BASELINE.json cfg1 (one 256x256 cascade,
// JONSWAP/TMA spectrum + 2D IFFT on the C# scalar CPU path) or any N / cascade count, timed with
// Stopwatch: the scalar single-thread run (primary) and Parallel.For over the host's cores
// (secondary, core count recorded). Median of >= 3 frames after 1 warm-up. One JSON line, the
// shape of bench.py's cpu_baseline object.
//     dotnet run -c Release -- [n] [cascades] [frames]
// Compile-ready; not built here (no C# toolchain in this image or on the GPU box: bench.py
// times the C port oracle/ocean_oracle.c, the same op order, and labels it as the stand-in).
using System;
using System.Diagnostics;
using System.Linq;

namespace OceanHip
{
    public static class CpuOceanBench
    {
        // Assets/Scenes/Waves.unity:1305-1314 (params) and the cascades :1431-1435, :470-474, :1249-1253,
        // plus the unreferenced 4th (:1572-1576)
        static readonly CpuCascade[] Scene =
        {
            new CpuCascade { wavelength = 1530f, cutoffLow = 1e-10f, cutoffHigh = 1e12f, swell = 0.4f, fade = 0.1f },
            new CpuCascade { wavelength = 1000f, cutoffLow = 1e-7f, cutoffHigh = 1e7f, swell = 0.3f, fade = 0.2f },
            new CpuCascade { wavelength = 201f, cutoffLow = 1e-5f, cutoffHigh = 1e6f, swell = 0.1f, fade = 0.1f },
            new CpuCascade { wavelength = 34f, cutoffLow = 0.001f, cutoffHigh = 10f, swell = 0.4f, fade = 0.1f },
        };

        static double MedianFrameSeconds(CpuOcean ocean, int frames, float t0)
        {
            ocean.CalculateWavesTexturesAtTime(t0);  // warm-up (JIT, pages, thread pool)
            var ts = new double[frames];
            for (int f = 0; f < frames; f++)
            {
                var sw = Stopwatch.StartNew();
                ocean.CalculateWavesTexturesAtTime(t0 + (f + 1) / 60.0f);
                ts[f] = sw.Elapsed.TotalSeconds;
            }
            return ts.OrderBy(x => x).ElementAt(frames / 2);
        }

        public static int Main(string[] args)
        {
            int n = args.Length > 0 ? int.Parse(args[0]) : 256;
            int cascades = args.Length > 1 ? int.Parse(args[1]) : 1;
            int frames = Math.Max(3, args.Length > 2 ? int.Parse(args[2]) : 3);
            var prm = new CpuOceanParams { windSpeed = 8f, windDirX = 1f, windDirY = -1f, gravity = 9.81f, fetch = 50000f,
                                           depth = 2560f };
            var ocean = new CpuOcean(n, prm, Scene.Take(cascades).ToArray(), CpuOcean.GenerateRandomNoiseTexture(n, 20251121));
            double single = MedianFrameSeconds(ocean, frames, 0f);
            int cores = Environment.ProcessorCount;
            ocean.Threads = cores;
            double multi = MedianFrameSeconds(ocean, frames, 1f);
            Console.WriteLine(
                $"{{\"value\": {1.0 / single:F4}, \"unit\": \"frames/s\", \"cores\": 1, \"kind\": \"port\", " +
                $"\"sample\": \"median of {frames} frames after 1 warm-up, {cascades} x {n}^2, C# scalar (CpuOcean.cs)\", " +
                $"\"multicore\": {{\"value\": {1.0 / multi:F4}, \"cores\": {cores}, \"sample\": \"Parallel.For over rows\"}}}}");
            return 0;
        }
    }
}
