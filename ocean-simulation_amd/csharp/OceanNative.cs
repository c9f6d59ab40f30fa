// P/Invoke binding of liboceanhip.so (include/ocean/ocean.h) for the reference's
// C# host (Unity / Mono / .NET).  Compile-ready; not built in this repository's CI
// (no C# toolchain in the build image).  Every struct is blittable and laid out
// exactly as the C declaration; every call returns OceanStatus (0 = OK).
using System;
using System.Runtime.InteropServices;

namespace OceanHip
{
    public enum OceanStatus : int
    {
        Ok = 0,
        InvalidArg = -1,
        Unsupported = -2,
        State = -3,
        Device = -4,
        OutOfMemory = -5,
    }

    [Flags]
    public enum OceanFlags : uint
    {
        None = 0,
        DisplacementOnly = 0x1,  // 2 planes -> DISP only
        Normals = 0x2,           // also write the per-cascade NORMAL texture
        Unfused = 0x4,           // reference-shaped schedule: evolve -> 4 x IFFT -> fill
        Mips = 0x8,              // DERIV / TURB mip chains regenerated every step (GenerateMips)
    }

    public enum OceanTexture : int
    {
        Noise = 0, H0 = 1, Waves = 2,
        Plane0 = 3, Plane1 = 4, Plane2 = 5, Plane3 = 6,   // DxDz, DyDxz, DyxDyz, DxxDzz
        Displacement = 7, Derivatives = 8, Turbulence = 9, Normal = 10,
    }

    // WaterBody.cs:10-14
    [StructLayout(LayoutKind.Sequential)]
    public struct OceanParams
    {
        public float windSpeed, windDirX, windDirY, gravity, fetch, depth;
    }

    // WaterCascade.cs:10-24
    [StructLayout(LayoutKind.Sequential)]
    public struct OceanCascade
    {
        public float wavelength, cutoffLow, cutoffHigh, swell, fade;
    }

    public static class OceanNative
    {
        public const int AbiVersion = 4;  // OCEAN_ABI_VERSION of the header this binding follows
        const string Lib = "oceanhip";  // liboceanhip.so next to the managed assembly / on LD_LIBRARY_PATH

        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_create(int device, int n, int nCascades, int nTiles, OceanFlags flags, out IntPtr ctx);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern void ocean_destroy(IntPtr ctx);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_set_params(IntPtr ctx, ref OceanParams p, [In] OceanCascade[] cascades);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_set_noise(IntPtr ctx, int tile, [In] float[] rg);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_generate_noise(IntPtr ctx, ulong seed);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_generate_noise_device(IntPtr ctx, ulong seed);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_init_spectrum(IntPtr ctx);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_reset_foam(IntPtr ctx);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_step(IntPtr ctx, float time);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_evolve(IntPtr ctx, float time);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_ifft2d(IntPtr ctx, int planeMask);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_fill(IntPtr ctx);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_read(IntPtr ctx, OceanTexture tex, int tile, int cascade, [Out] float[] dst, UIntPtr bytes);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_write(IntPtr ctx, OceanTexture tex, int tile, int cascade, [In] float[] src, UIntPtr bytes);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_get_device_ptr(IntPtr ctx, OceanTexture tex, out IntPtr ptr, out UIntPtr bytes);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_get_stream(IntPtr ctx, out IntPtr stream);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_synchronize(IntPtr ctx);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_set_kernel_timing(IntPtr ctx, int enable);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_kernel_stats(IntPtr ctx, int kind, out double totalMs, out long launches);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_kernel_name(IntPtr ctx, int kind, [Out] byte[] buf, UIntPtr len);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_step_bytes(IntPtr ctx, out ulong passA, out ulong passB);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_set_column_band(IntPtr ctx, int xBegin, int xCount);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_set_column_parity(IntPtr ctx, int parity);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_read_mip(IntPtr ctx, OceanTexture tex, int tile, int cascade, int level, [Out] float[] dst, UIntPtr bytes);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_get_mip_ptr(IntPtr ctx, OceanTexture tex, int level, out IntPtr ptr, out UIntPtr sliceStride);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_sample_world(IntPtr ctx, int tile, [In] float[] points, int count, [Out] float[] output);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_sample_world_device(IntPtr ctx, int tile, IntPtr points, int count, IntPtr output);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_read_async(IntPtr ctx, OceanTexture tex, int tile, int cascade, IntPtr dst, UIntPtr bytes, out IntPtr request);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern int ocean_readback_status(IntPtr request);   // 1 done, 0 pending, < 0 error (hasError)
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_readback_wait(IntPtr request);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern void ocean_readback_release(IntPtr request);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_readback_copy_ms(IntPtr request, out float ms);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_read_height_async(IntPtr ctx, int tile, int cascade, IntPtr dst, UIntPtr bytes, out IntPtr request);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_set_readback_timing(IntPtr ctx, int enable);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern OceanStatus ocean_host_alloc(UIntPtr bytes, out IntPtr ptr);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern void ocean_host_free(IntPtr ptr);
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        static extern IntPtr ocean_last_error();
        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]
        public static extern int ocean_abi_version();

        public static string LastError() => Marshal.PtrToStringAnsi(ocean_last_error()) ?? "";

        public static void Check(OceanStatus s, string where)
        {
            if (s != OceanStatus.Ok) throw new InvalidOperationException($"{where} failed ({s}): {LastError()}");
        }
    }
}
