// WaterBody-shaped facade over liboceanhip.so: the same public surface as
// Assets/Scripts/Water/WaterBody.cs (fields :10-33, CalculateWavesTexturesAtTime
// :180, GetWaterHeight :195, Awake :211, Update :284, OnDisable :300), with the
// GPU work done by the MI355X library instead of ComputeShader.Dispatch.
// Engine-free (no UnityEngine types) so it also runs in a plain .NET host; a
// Unity MonoBehaviour can own one of these and forward its lifecycle calls.
// Compile-ready; not built here (no C# toolchain in the build image).
using System;

namespace OceanHip
{
    public sealed class WaterCascadeDesc  // WaterCascade.cs:10-24
    {
        public float wavelength = 10.0f, cutoffHigh = 5.0f, cutoffLow = 0.0001f, swell = 0.4f, fade = 0.1f;
    }

    // What Update reads back every frame (ocean.h ocean_read_height_async): the height channel alone,
    // all GetWaterHeight reads (the reference's buoyancyData is private, WaterBody.cs:58, and .g is its
    // only use, :208), or the whole RGBA displacement slice as the reference requests it.
    public enum Readback { Height, Rgba }

    public sealed class WaterBodyNative : IDisposable
    {
        // Ocean parameters (WaterBody.cs:10-14) and texture size (:29)
        public float windSpeed = 1.0f;
        public float windDirectionX = 1.0f, windDirectionY = 1.0f;
        public float gravity = 9.81f;
        public float fetch = 1.0f;
        public float depth = 4.0f;
        public int texturesSize = 256;
        public WaterCascadeDesc[] cascades = { new WaterCascadeDesc() };
        public int device = 0;
        public ulong seed = 20251121;   // the reference's UnityEngine.Random is unseeded; this library's generator is
        public Readback readback = Readback.Height;  // set before Awake

        IntPtr ctx = IntPtr.Zero;
        float[] buoyancyData;           // displacement slice 0 (WaterBody.cs:58, :295): [y][x] heights, or RGBA [y][x][4]
        int Floats => texturesSize * texturesSize * (readback == Readback.Height ? 1 : 4);  // per readback slice

        public void Awake()
        {
            // the rules this facade relies on (ocean.h: ABI 4, no call moves the caller's current device)
            if (OceanNative.ocean_abi_version() != OceanNative.AbiVersion)
                throw new InvalidOperationException("liboceanhip ABI " + OceanNative.ocean_abi_version() + ", expected " +
                                                    OceanNative.AbiVersion);
            OceanNative.Check(OceanNative.ocean_create(device, texturesSize, cascades.Length, 1, OceanFlags.Mips, out ctx),
                              "ocean_create");
            ApplyParams();
            OceanNative.Check(OceanNative.ocean_generate_noise(ctx, seed), "ocean_generate_noise");
            OceanNative.Check(OceanNative.ocean_init_spectrum(ctx), "ocean_init_spectrum");
            // readback ring: MaxReadbacksInFlight pinned slices allocated once, reused by every
            // request and freed only in Dispose (hipHostFree synchronizes the device: a free per
            // request would make each Update wait for the frame it just queued)
            int bytes = Floats * sizeof(float);
            for (int i = 0; i < MaxReadbacksInFlight; i++)
            {
                OceanNative.Check(OceanNative.ocean_host_alloc((UIntPtr)bytes, out var b), "ocean_host_alloc");
                ring.Add(b);
                idle.Push(b);
            }
        }

        void ApplyParams()
        {
            var p = new OceanParams { windSpeed = windSpeed, windDirX = windDirectionX, windDirY = windDirectionY,
                                      gravity = gravity, fetch = fetch, depth = depth };
            var cs = new OceanCascade[cascades.Length];
            for (int i = 0; i < cascades.Length; i++)
                cs[i] = new OceanCascade { wavelength = cascades[i].wavelength, cutoffLow = cascades[i].cutoffLow,
                                           cutoffHigh = cascades[i].cutoffHigh, swell = cascades[i].swell,
                                           fade = cascades[i].fade };
            OceanNative.Check(OceanNative.ocean_set_params(ctx, ref p, cs), "ocean_set_params");
        }

        // The commented OnValidate of WaterBody.cs:324-337: parameter change -> spectrum re-init
        // (the foam accumulator carries over, as there).
        public void OnValidate()
        {
            if (ctx == IntPtr.Zero) return;
            ApplyParams();
            OceanNative.Check(OceanNative.ocean_init_spectrum(ctx), "ocean_init_spectrum");
        }

        public void CalculateWavesTexturesAtTime(float time) =>
            OceanNative.Check(OceanNative.ocean_step(ctx, time), "ocean_step");

        // WaterBody.Update (:284-297): step, then issue a new asynchronous request of the
        // displacement slice 0 EVERY frame (AsyncGPUReadback.Request, :288); requests
        // complete in order and each completed one refreshes buoyancyData, as the
        // reference's callback does (:292-295).  Requests land in slots of a pinned ring.
        const int MaxReadbacksInFlight = 4;  // ring slots; the reference's request queue is engine-managed.
                                             // 2-4 in flight keep the 16 MiB copies back to back beside the
                                             // frames; 8 stretch each copy 2.5x (DESIGN.md section 1)
        readonly System.Collections.Generic.Queue<(IntPtr req, IntPtr buf)> readbacks =
            new System.Collections.Generic.Queue<(IntPtr req, IntPtr buf)>();
        readonly System.Collections.Generic.List<IntPtr> ring = new System.Collections.Generic.List<IntPtr>();
        readonly System.Collections.Generic.Stack<IntPtr> idle = new System.Collections.Generic.Stack<IntPtr>();

        void Complete((IntPtr req, IntPtr buf) r, bool wait)
        {
            int n = Floats;
            int st = wait ? (OceanNative.ocean_readback_wait(r.req) == OceanStatus.Ok ? 1 : -1)
                          : OceanNative.ocean_readback_status(r.req);
            if (st == 1)
            {
                buoyancyData ??= new float[n];
                System.Runtime.InteropServices.Marshal.Copy(r.buf, buoyancyData, 0, n);
            }                                              // st < 0: request.hasError, data dropped
            OceanNative.ocean_readback_release(r.req);
            idle.Push(r.buf);                              // slot back to the ring
        }

        public void Update(float time)
        {
            CalculateWavesTexturesAtTime(time);
            while (readbacks.Count > 0 && OceanNative.ocean_readback_status(readbacks.Peek().req) != 0)
                Complete(readbacks.Dequeue(), false);
            if (idle.Count == 0) Complete(readbacks.Dequeue(), true);  // every slot in flight: wait for the oldest
            var buf = idle.Pop();
            var bytes = (UIntPtr)(Floats * sizeof(float));
            IntPtr req;
            var st = readback == Readback.Height
                         ? OceanNative.ocean_read_height_async(ctx, 0, 0, buf, bytes, out req)
                         : OceanNative.ocean_read_async(ctx, OceanTexture.Displacement, 0, 0, buf, bytes, out req);
            if (st != OceanStatus.Ok) { idle.Push(buf); OceanNative.Check(st, "readback request"); }
            readbacks.Enqueue((req, buf));
        }

        public void WaitForReadbacks()
        {
            while (readbacks.Count > 0) Complete(readbacks.Dequeue(), true);
        }

        // WaterBody.cs:195-209, including the mapping over [-texturesSize/2, texturesSize/2].
        public float GetWaterHeight(float worldX, float worldZ)
        {
            if (buoyancyData == null) return 0f;
            float InverseLerp(float a, float b, float v) => a == b ? 0f : Math.Clamp((v - a) / (b - a), 0f, 1f);
            float u = InverseLerp(-texturesSize / 2, texturesSize / 2, worldX);
            float v = InverseLerp(-texturesSize / 2, texturesSize / 2, worldZ);
            int x = Math.Clamp((int)(u * texturesSize), 0, texturesSize - 1);
            int y = Math.Clamp((int)(v * texturesSize), 0, texturesSize - 1);
            int t = y * texturesSize + x;
            return readback == Readback.Height ? buoyancyData[t] : buoyancyData[t * 4 + 1];  // .g = Dy
        }

        // What Water.shader reads at world positions (Water.shader:314-348): points are
        // (x, z, lod) triples; per point 12 floats: summed displacement + turbulence,
        // summed derivatives, normal (ocean.h ocean_sample_world).
        public float[] SampleWorld(float[] points)
        {
            var output = new float[points.Length / 3 * 12];
            OceanNative.Check(OceanNative.ocean_sample_world(ctx, 0, points, points.Length / 3, output), "ocean_sample_world");
            return output;
        }

        // Texture-out contract: device pointers for same-process renderers (WaterBody.cs:277-281).
        public IntPtr DeviceTexture(OceanTexture tex, out ulong bytes)
        {
            OceanNative.Check(OceanNative.ocean_get_device_ptr(ctx, tex, out var p, out var b), "ocean_get_device_ptr");
            bytes = (ulong)b;
            return p;
        }

        public void OnDisable() => Dispose();

        public void Dispose()
        {
            while (readbacks.Count > 0) OceanNative.ocean_readback_release(readbacks.Dequeue().req);
            foreach (var b in ring) OceanNative.ocean_host_free(b);
            ring.Clear();
            idle.Clear();
            if (ctx != IntPtr.Zero) OceanNative.ocean_destroy(ctx);
            ctx = IntPtr.Zero;
        }
    }
}
