// CpuOcean -- the scalar C# CPU baseline of north_star ("a C# scalar CPU re-implementation of
// the same path"; BASELINE.json cfg1: one 256x256 cascade on the C# scalar CPU path).
//
// It runs the reference's per-frame path on the host in the reference's own operation order,
// fp32 throughout (System.MathF), one element at a time:
//   noise           Assets/Scripts/Water/WaterBody.cs:71-100 (Marsaglia polar, x-outer /
//                   y-inner, g1 then g2) over this library's documented seeded uniform source
//                   (xorshift128 seeded by splitmix64; UnityEngine.Random is unseeded and
//                   closed, include/ocean/ocean.h ocean_generate_noise) -- the same texture the
//                   GPU library's ocean_generate_noise uploads, bit for bit
//   init spectrum   InitialSpectrum.compute:33-129, conjugate :135-143
//   evolve          TimeDependentSpectrum.compute:20-47 (packed planes :42-45)
//   IFFT            IFFT.cs:24-94 + IFFT.compute:37-78: the twiddle/index table, log2 N
//                   horizontal + log2 N vertical radix-2 ping-pong passes, the permute
//   fill / foam     ResultTexturesFiller.compute:16-34
//   frame           WaterBody.CalculateWavesTexturesAtTime, WaterBody.cs:180-193 (no mips)
// Engine-free: no UnityEngine types, so it runs in a plain .NET host (CpuOceanBench.cs).
// Compile-ready; not built here (no C# toolchain in this image or on the GPU box). The
// measured stand-in with the same op order is the C port oracle/ocean_oracle.c (bench.py
// cpu_baseline), which this file follows function for function.
using System;
using System.Threading.Tasks;

namespace OceanHip
{
    public struct CpuOceanParams  // WaterBody.cs:10-14
    {
        public float windSpeed, windDirX, windDirY, gravity, fetch, depth;
    }

    public struct CpuCascade  // WaterCascade.cs:10-24
    {
        public float wavelength, cutoffLow, cutoffHigh, swell, fade;
    }

    public sealed class CpuOcean
    {
        const float PI = 3.14159265f;                       // InitialSpectrum.compute:8, IFFT.compute:7
        const float FoamDecay = 0.135335283236612691894f;   // exp(-2), ResultTexturesFiller.compute:29-30

        public readonly int N, C, Planes;                   // Planes: 4 full, 2 displacement only
        public readonly float[] Noise;                      // float2 [N][N]
        public readonly float[] H0, Waves;                  // float4 [C][N][N]
        public readonly float[][] Plane;                    // 4 x float2 [C][N][N]: DxDz, DyDxz, DyxDyz, DxxDzz
        public readonly float[] Displacement, Derivatives, Turbulence;  // float4 [C][N][N]
        readonly float[] pingPong, table;
        readonly int logN;
        readonly CpuOceanParams p;
        readonly CpuCascade[] cascades;
        /// Parallel.For over rows in the per-frame loops (the secondary, multi-core figure of
        /// SURVEY.md 8d); 1 = the scalar single-thread baseline. Every element is computed by
        /// the same expression either way, so the result does not depend on it.
        public int Threads = 1;

        public CpuOcean(int n, CpuOceanParams prm, CpuCascade[] cs, float[] noise, bool displacementOnly = false)
        {
            if (n < 2 || (n & (n - 1)) != 0) throw new ArgumentException("n must be a power of two");
            N = n; C = cs.Length; Planes = displacementOnly ? 2 : 4;
            p = prm; cascades = cs;
            while ((1 << logN) < n) logN++;
            Noise = noise;
            int tex = C * n * n;
            H0 = new float[tex * 4]; Waves = new float[tex * 4];
            Plane = new float[4][];
            for (int i = 0; i < 4; i++) Plane[i] = new float[tex * 2];
            pingPong = new float[tex * 2];
            Displacement = new float[tex * 4];
            Derivatives = displacementOnly ? null : new float[tex * 4];
            Turbulence = displacementOnly ? null : new float[tex * 4];
            table = new float[logN * n * 4];
            PrecomputeTwiddleFactorsAndInputIndices();
            CalculateInitialSpectrumTextures();
        }

        // ---------------------------------------------------------------- noise
        // WaterBody.cs:71-100 over xorshift128 seeded by splitmix64 (U = (u32 >> 8) * 2^-24).
        public static float[] GenerateRandomNoiseTexture(int n, ulong seed)
        {
            ulong x = seed;
            ulong SplitMix()
            {
                unchecked
                {
                    ulong z = (x += 0x9E3779B97F4A7C15UL);
                    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9UL;
                    z = (z ^ (z >> 27)) * 0x94D049BB133111EBUL;
                    return z ^ (z >> 31);
                }
            }
            ulong a = SplitMix(), b = SplitMix();
            uint s0 = (uint)a, s1 = (uint)(a >> 32), s2 = (uint)b, s3 = (uint)(b >> 32);
            if ((s0 | s1 | s2 | s3) == 0) s0 = 1;
            float Uniform()
            {
                uint t = s0 ^ (s0 << 11);
                s0 = s1; s1 = s2; s2 = s3;
                s3 = s3 ^ (s3 >> 19) ^ t ^ (t >> 8);
                return (float)(s3 >> 8) * (1.0f / 16777216.0f);
            }
            float GenerateRandomNumber()  // :71-81
            {
                float v1, v2, s;
                do
                {
                    v1 = 2.0f * Uniform() - 1.0f;
                    v2 = 2.0f * Uniform() - 1.0f;
                    s = v1 * v1 + v2 * v2;
                } while (s >= 1.0f || s == 0.0f);
                s = MathF.Sqrt((-2.0f * MathF.Log(s)) / s);
                return v1 * s;
            }
            var noise = new float[n * n * 2];
            for (int i = 0; i < n; i++)      // :90-95, i = x outer
                for (int j = 0; j < n; j++)  // j = y inner
                {
                    float g1 = GenerateRandomNumber();
                    float g2 = GenerateRandomNumber();
                    noise[(j * n + i) * 2 + 0] = g1;
                    noise[(j * n + i) * 2 + 1] = g2;
                }
            return noise;
        }

        // -------------------------------------------------------- initial spectrum
        // The initial spectrum's transcendentals, each correctly rounded (double, one rounding), as the
        // oracle (oracle/ocean_oracle.c cr_*) and the HIP library evaluate them: h0 bit-exact across the three.
        static float CrPow(float a, float b) => (float)Math.Pow(a, b);
        static float CrExp(float a) => (float)Math.Exp(a);
        static float CrLog(float a) => (float)Math.Log(a);
        static float CrTanh(float a) => (float)Math.Tanh(a);
        static float CrCosh(float a) => (float)Math.Cosh(a);
        static float CrCos(float a) => (float)Math.Cos(a);
        static float CrAtan2(float a, float b) => (float)Math.Atan2(a, b);

        float AngularFrequency(float k) => MathF.Sqrt(p.gravity * k);  // InitialSpectrum.compute:33-35

        float TMACorrection(float w)  // :38-43
        {
            float wh = w * MathF.Sqrt(p.depth / p.gravity);
            if (wh <= 1.0f) return 0.5f * wh * wh;
            if (wh < 2.0f) return 1.0f - 0.5f * (2.0f - wh) * (2.0f - wh);
            return 1.0f;
        }

        float JONSWAP(float w, float wp)  // :47-56
        {
            float alpha = 0.076f * CrPow(MathF.Abs(p.windSpeed * p.windSpeed / (p.fetch * p.gravity)), 0.22f);
            float gamma = 3.3f;
            float sigma = w <= wp ? 0.07f : 0.09f;
            float d = w - wp;
            float r = CrExp(-(d * d) / (2.0f * sigma * sigma * wp * wp));
            return alpha * p.gravity * p.gravity / CrPow(w, 5.0f) * CrExp(-1.25f * CrPow(wp / w, 4.0f)) *
                   CrPow(MathF.Abs(gamma), r);
        }

        float SpreadPower(float w, float wp)  // :60-66
        {
            if (w < 1.05f * wp) return 6.97f * CrPow(MathF.Abs(w / wp), 4.06f);
            float peakSpeed = p.gravity / wp;
            float mu = -2.33f - 1.45f * (p.windSpeed / peakSpeed - 1.17f);
            return 9.77f * CrPow(MathF.Abs(w / wp), mu);
        }

        static float NormalizationFactor(float s)  // :69-74
        {
            float s2 = s * s, s3 = s2 * s;
            if (s <= 0.4f)
                return 0.09f * s3 + (CrPow(CrLog(2.0f), 2.0f) / PI - PI / 12.0f) * s2 + CrLog(2.0f) / PI * s +
                       1.0f / (2.0f * PI);
            return MathF.Sqrt(s) / (2.0f * MathF.Sqrt(PI)) + 1.0f / (16.0f * MathF.Sqrt(PI * s));
        }

        float DirectionalSpread(float w, float wp, float theta, float swell)  // :78-84
        {
            float s = SpreadPower(w, wp) + 16.0f * CrTanh(w / wp) * swell * swell;
            float len = MathF.Sqrt(p.windDirX * p.windDirX + p.windDirY * p.windDirY);  // normalize(_WindDirection)
            float windTheta = CrAtan2(p.windDirY / len, p.windDirX / len);
            return NormalizationFactor(s) * CrPow(MathF.Abs(CrCos(0.5f * (theta - windTheta))), 2.0f * s);
        }

        float FrequencyDerivative(float k, float w)  // :87-91
        {
            float th = CrTanh(MathF.Min(k * p.depth, 20.0f));
            float ch = CrCosh(k * p.depth);
            return p.gravity * (p.depth * k / ch / ch + th) / (w * 2.0f);
        }

        static float ShortWavesFade(float k, float fade) => CrExp(-fade * fade * k * k);  // :95-97

        // CalculateInitialSpectrumTextures (WaterBody.cs:171-178): :99-129 then :135-143.
        public void CalculateInitialSpectrumTextures()
        {
            int n = N, half = n / 2;
            float wp = 22.0f * CrPow(MathF.Abs(p.gravity * p.gravity / (p.windSpeed * p.fetch)), 0.3333f);  // :118
            for (int c = 0; c < C; c++)
            {
                float dk = 2.0f * PI / cascades[c].wavelength;  // :110
                for (int y = 0; y < n; y++)
                    for (int x = 0; x < n; x++)
                    {
                        int t = y * n + x, o = ((c * n + y) * n + x) * 4;
                        float g1 = Noise[t * 2], g2 = Noise[t * 2 + 1];
                        float kx = (x - half) * dk, kz = (y - half) * dk;
                        float kmag = MathF.Sqrt(kx * kx + kz * kz);
                        if (kmag >= cascades[c].cutoffLow && kmag <= cascades[c].cutoffHigh)
                        {
                            float kangle = CrAtan2(kz, kx);
                            float w = AngularFrequency(kmag);
                            float amp = MathF.Sqrt(2.0f * TMACorrection(w) * JONSWAP(w, wp) *
                                                   DirectionalSpread(w, wp, kangle, cascades[c].swell) *
                                                   ShortWavesFade(kmag, cascades[c].fade) * FrequencyDerivative(kmag, w) /
                                                   kmag * dk * dk);
                            H0[o] = g1 / 2.0f * amp; H0[o + 1] = g2 / 2.0f * amp; H0[o + 2] = 0; H0[o + 3] = 0;
                            Waves[o] = kx; Waves[o + 1] = 1.0f / kmag; Waves[o + 2] = kz; Waves[o + 3] = w;
                        }
                        else
                        {
                            H0[o] = H0[o + 1] = H0[o + 2] = H0[o + 3] = 0;
                            Waves[o] = kx; Waves[o + 1] = 1.0f; Waves[o + 2] = kz; Waves[o + 3] = 0;
                        }
                    }
                // CalculateConjugatedInitialSpectrumTextures (:135-143): .zw = conj h0(-k); only .xy is read
                for (int y = 0; y < n; y++)
                    for (int x = 0; x < n; x++)
                    {
                        int o = ((c * n + y) * n + x) * 4, m = ((c * n + (n - y) % n) * n + (n - x) % n) * 4;
                        H0[o + 2] = H0[m];
                        H0[o + 3] = -H0[m + 1];
                    }
            }
        }

        // ------------------------------------------------------------------ evolve
        // TimeDependentSpectrum.compute:20-47
        void CalculateTimeDependentComplexAmplitudesAndDerivatives(float t)
        {
            int rowsTotal = C * N;
            Action<int> row = r =>
            {
                for (int i = r * N; i < (r + 1) * N; i++)
                {
                    int q = i * 4;
                    float phase = Waves[q + 3] * t;
                    float ex = MathF.Cos(phase), ey = MathF.Sin(phase);
                    float hx = (H0[q] * ex - H0[q + 1] * ey) + (H0[q + 2] * ex - H0[q + 3] * (-ey));
                    float hy = (H0[q] * ey + H0[q + 1] * ex) + (H0[q + 2] * (-ey) + H0[q + 3] * ex);
                    float ihx = -hy, ihy = hx;
                    float kx = Waves[q], ik = Waves[q + 1], kz = Waves[q + 2];
                    float ydxX = ihx * kx, ydxY = ihy * kx, ydzX = ihx * kz, ydzY = ihy * kz;
                    float dxX = ydxX * ik, dxY = ydxY * ik, dzX = ydzX * ik, dzY = ydzY * ik;
                    float auxX = -hx * ik, auxY = -hy * ik;
                    float dxxX = auxX * kx * kx, dxxY = auxY * kx * kx;
                    float dzzX = auxX * kz * kz, dzzY = auxY * kz * kz;
                    float dzxX = auxX * kx * kz, dzxY = auxY * kx * kz;
                    int o = i * 2;
                    Plane[0][o] = dxX - dzY; Plane[0][o + 1] = dxY + dzX;     // DxDz   (:42)
                    Plane[1][o] = hx - dzxY; Plane[1][o + 1] = hy + dzxX;     // DyDxz  (:43)
                    if (Planes == 4)
                    {
                        Plane[2][o] = ydxX - ydzY; Plane[2][o + 1] = ydxY + ydzX;  // DyxDyz (:44)
                        Plane[3][o] = dxxX - dzzY; Plane[3][o + 1] = dxxY + dzzX;  // DxxDzz (:45)
                    }
                }
            };
            For(rowsTotal, row);
        }

        // -------------------------------------------------------------------- IFFT
        // PrecomputeTwiddleFactorsAndInputIndices (IFFT.compute:37-45) -> float4 [log2 N][N]
        void PrecomputeTwiddleFactorsAndInputIndices()
        {
            float multY = 2.0f * PI * 1.0f / N;
            for (int s = 0; s < logN; s++)
                for (int y = 0; y < N / 2; y++)
                {
                    int b = N >> (s + 1);
                    int i = (2 * b * (y / b) + y % b) % N;
                    float arg = -multY * ((y / b) * b);
                    float tx = MathF.Cos(arg), ty = MathF.Sin(arg);
                    int a = (s * N + y) * 4, bb = (s * N + y + N / 2) * 4;
                    table[a] = tx; table[a + 1] = ty; table[a + 2] = i; table[a + 3] = i + b;
                    table[bb] = -tx; table[bb + 1] = -ty; table[bb + 2] = i; table[bb + 3] = i + b;
                }
        }

        // InverseFastFourierTransform (IFFT.cs:66-94), in place on one float2 [C][N][N] plane array
        public void InverseFastFourierTransform(float[] input)
        {
            int n = N;
            bool pp = false;
            for (int dir = 0; dir < 2; dir++)
                for (int s = 0; s < logN; s++)
                {
                    float[] src = pp ? pingPong : input, dst = pp ? input : pingPong;
                    int stage = s, d0 = dir;
                    For(C * n, r =>
                    {
                        int c = r / n, y = r % n;
                        for (int x = 0; x < n; x++)
                        {
                            // HorizontalStepIFFT (:48-57) indexes the table by x, VerticalStepIFFT (:60-69) by y
                            int d = (stage * n + (d0 == 0 ? x : y)) * 4;
                            float wx = table[d], wy = -table[d + 1];  // conjugated twiddle: the inverse
                            int i0 = (int)table[d + 2], i1 = (int)table[d + 3];
                            int a0 = d0 == 0 ? (c * n + y) * n + i0 : (c * n + i0) * n + x;
                            int a1 = d0 == 0 ? (c * n + y) * n + i1 : (c * n + i1) * n + x;
                            float bx = src[a1 * 2], by = src[a1 * 2 + 1];
                            int o = ((c * n + y) * n + x) * 2;
                            dst[o] = src[a0 * 2] + (wx * bx - wy * by);
                            dst[o + 1] = src[a0 * 2 + 1] + (wx * by + wy * bx);
                        }
                    });
                    pp = !pp;
                }
            // 2 log2 N passes: the result is back in `input`. Permute (IFFT.compute:73-78).
            For(C * n, r =>
            {
                int y = r % n;
                for (int x = 0; x < n; x++)
                {
                    float sgn = 1.0f - 2.0f * ((x + y) % 2);
                    int o = (r * n + x) * 2;
                    input[o] *= sgn;
                    input[o + 1] *= sgn;
                }
            });
        }

        // -------------------------------------------------------------------- fill
        // FillResultTextures (ResultTexturesFiller.compute:16-34)
        void FillResultTextures()
        {
            For(C * N, r =>
            {
                for (int i = r * N; i < (r + 1) * N; i++)
                {
                    int o = i * 4, q = i * 2;
                    Displacement[o] = Plane[0][q];
                    Displacement[o + 1] = Plane[1][q];
                    Displacement[o + 2] = Plane[0][q + 1];
                    Displacement[o + 3] = 1.0f;  // alpha unspecified in the reference (float3 store)
                    if (Planes != 4) continue;
                    Derivatives[o] = Plane[2][q]; Derivatives[o + 1] = Plane[2][q + 1];
                    Derivatives[o + 2] = Plane[3][q]; Derivatives[o + 3] = Plane[3][q + 1];
                    float jacobian = (1.0f + Plane[3][q]) * (1.0f + Plane[3][q + 1]) - Plane[1][q + 1] * Plane[1][q + 1];
                    float foam = Turbulence[o];
                    foam *= FoamDecay;
                    if (foam < jacobian) foam += jacobian;
                    Turbulence[o] = Turbulence[o + 1] = Turbulence[o + 2] = Turbulence[o + 3] = foam;
                }
            });
        }

        // ------------------------------------------------------------------- frame
        // CalculateWavesTexturesAtTime (WaterBody.cs:180-193), mips excluded (SURVEY.md 8d)
        public void CalculateWavesTexturesAtTime(float time)
        {
            CalculateTimeDependentComplexAmplitudesAndDerivatives(time);
            for (int i = 0; i < Planes; i++) InverseFastFourierTransform(Plane[i]);
            FillResultTextures();
        }

        void For(int count, Action<int> body)
        {
            if (Threads <= 1)
            {
                for (int i = 0; i < count; i++) body(i);
                return;
            }
            Parallel.For(0, count, new ParallelOptions { MaxDegreeOfParallelism = Threads }, body);
        }
    }
}
