"""CPU test that the C# P/Invoke binding (ocean-simulation_amd/csharp/OceanNative.cs) matches the C ABI
(include/ocean/ocean.h): the north star's host is C#, and no C# compiler exists here or on the GPU box, so
this is what keeps the binding true.  Checked against the header text:
  - every header entry point has exactly one DllImport of the same name, with the same arity and
    a marshalling-compatible type per parameter and for the return value, and there are no others;
  - OceanParams / OceanCascade: LayoutKind.Sequential, the header struct's fields in the same order;
  - the OceanStatus / OceanFlags / OceanTexture values equal the header's macros and enum;
  - OceanNative.AbiVersion == OCEAN_ABI_VERSION, and WaterBodyNative.Awake refuses any other library version.
The checker must also catch a broken binding: mutants (a dropped parameter, swapped struct fields, a wrong
version, a renamed or missing entry) each have to be reported."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ocean", "ocean.h")
NATIVE = os.path.join(ROOT, "ocean-simulation_amd", "csharp", "OceanNative.cs")
FACADE = os.path.join(ROOT, "ocean-simulation_amd", "csharp", "WaterBodyNative.cs")

# C parameter / return type (normalised: no const, no names) -> the C# types that marshal to it
COMPAT = {
    "ocean_ctx*": {"IntPtr"},
    "ocean_ctx**": {"out IntPtr"},
    "ocean_readback*": {"IntPtr"},
    "ocean_readback**": {"out IntPtr"},
    "int": {"int", "OceanStatus", "OceanTexture"},
    "uint32_t": {"uint", "OceanFlags"},
    "uint64_t": {"ulong"},
    "float": {"float"},
    "size_t": {"UIntPtr"},
    "void": {"void"},
    "void*": {"IntPtr", "[Out] float[]", "[In] float[]"},  # a pinned blittable array for a texel buffer
    "float*": {"IntPtr", "[Out] float[]", "[In] float[]", "float[]"},
    "char*": {"IntPtr", "[Out] byte[]"},
    "double*": {"out double"},
    "long long*": {"out long"},
    "uint64_t*": {"out ulong"},
    "size_t*": {"out UIntPtr"},
    "void**": {"out IntPtr"},
    "float*out": {"out float"},
    "ocean_params*": {"ref OceanParams"},
    "ocean_cascade*": {"[In] OceanCascade[]", "OceanCascade[]"},
}


def _strip_c(text):
    return re.sub(r"/\*.*?\*/", "", text, flags=re.S)


def header_prototypes(h):
    """name -> (return type, [parameter types]) from ocean.h."""
    protos = {}
    for ret, name, args in re.findall(r"^\s*((?:const\s+)?[a-z_0-9 ]+?\s*\**)\s*\b(ocean_[a-z0-9_]+)\s*\(([^)]*)\)\s*;",
                                      _strip_c(h), flags=re.M):
        params = []
        for a in [x.strip() for x in args.split(",")]:
            if a in ("", "void"):
                continue
            a = re.sub(r"\bconst\b", "", a)
            stars = a.count("*")
            words = a.replace("*", " ").split()
            base = " ".join(words[:-1]) if len(words) > 1 else words[0]  # drop the parameter name
            params.append(base + "*" * stars)
        r = re.sub(r"\bconst\b", "", ret).replace(" ", "")
        protos[name] = (r, params)
    return protos


def header_struct(h, name):
    body = re.search(r"typedef struct " + name + r"\s*\{(.*?)\}\s*" + name + ";", _strip_c(h), flags=re.S).group(1)
    return [(t, n) for t, n in re.findall(r"(\w+)\s+(\w+);", body)]


def cs_imports(cs):
    """name -> [(return type, [parameter types])] of every DllImport in OceanNative.cs."""
    out = {}
    for ret, name, args in re.findall(r"\[DllImport\([^\]]*\)\]\s*(?:public\s+)?static\s+extern\s+(\w+)\s+(ocean_\w+)\s*"
                                      r"\(([^)]*)\)\s*;", cs):
        params = []
        for a in [x.strip() for x in args.split(",") if x.strip()]:
            words = a.split()
            params.append(" ".join(words[:-1]))  # drop the parameter name
        out.setdefault(name, []).append((ret, params))
    return out


def cs_struct(cs, name):
    m = re.search(r"\[StructLayout\(LayoutKind\.Sequential\)\]\s*public struct " + name + r"\s*\{(.*?)\}", cs, flags=re.S)
    if not m:
        return None
    fields = []
    for typ, names in re.findall(r"public\s+(\w+)\s+([^;]+);", m.group(1)):
        fields += [(typ, n.strip()) for n in names.split(",")]
    return fields


def cs_enum(cs, name):
    body = re.search(r"public enum " + name + r"\s*:\s*\w+\s*\{(.*?)\}", cs, flags=re.S).group(1)
    body = re.sub(r"//[^\n]*", "", body)
    return {k: int(v, 0) for k, v in re.findall(r"(\w+)\s*=\s*(-?\w+)", body)}


def _norm(name):
    return name.replace("_", "").lower()


def check_binding(h, cs, facade):
    problems = []
    protos, imports = header_prototypes(h), cs_imports(cs)
    for name, (ret, params) in sorted(protos.items()):
        if name not in imports:
            problems.append(f"{name}: no DllImport")
            continue
        if len(imports[name]) != 1:
            problems.append(f"{name}: {len(imports[name])} DllImports")
        cret, cparams = imports[name][0]
        if cret not in COMPAT.get(ret, set()) and not (ret == "char*" and cret == "IntPtr"):
            problems.append(f"{name}: returns {cret}, header {ret}")
        if len(cparams) != len(params):
            problems.append(f"{name}: {len(cparams)} parameters, header {len(params)}")
            continue
        for i, (c, cc) in enumerate(zip(params, cparams)):
            ok = COMPAT.get(c, set()) | (COMPAT["float*out"] if c == "float*" else set())
            if cc not in ok:
                problems.append(f"{name} parameter {i}: C# {cc!r} for C {c!r}")
    for extra in sorted(set(imports) - set(protos)):
        problems.append(f"{extra}: DllImport of no header entry")
    for cname, csname in (("ocean_params", "OceanParams"), ("ocean_cascade", "OceanCascade")):
        hf, cf = header_struct(h, cname), cs_struct(cs, csname)
        if cf is None:
            problems.append(f"{csname}: not a LayoutKind.Sequential struct")
            continue
        if [(t, _norm(n)) for t, n in hf] != [(t, _norm(n)) for t, n in cf]:
            problems.append(f"{csname} fields {cf} != header {hf}")
    hs = _strip_c(h)
    status = {k: int(v) for k, v in re.findall(r"#define OCEAN_(OK|E_\w+)\s+\(?(-?\d+)\)?", hs)}
    if {_norm(k.replace("E_", "")): v for k, v in status.items()} != {_norm(k): v for k, v in cs_enum(cs, "OceanStatus").items()}:
        problems.append("OceanStatus values differ from the header's OCEAN_OK / OCEAN_E_*")
    flags = {k: int(v, 16) for k, v in re.findall(r"#define OCEAN_F_(\w+)\s+(0x[0-9a-fA-F]+)u", hs)}
    csf = {k: v for k, v in cs_enum(cs, "OceanFlags").items() if k != "None"}
    if {_norm(k) for k in flags} != {_norm(k) for k in csf} or \
            any(csf[k] != flags[f] for k in csf for f in flags if _norm(f) == _norm(k)):
        problems.append("OceanFlags differ from the header's OCEAN_F_*")
    tex = {k: int(v) for k, v in re.findall(r"OCEAN_TEX_(\w+)\s*=\s*(\d+)", hs)}
    cst = cs_enum(cs, "OceanTexture")
    if sorted(tex.values()) != sorted(cst.values()) or len(tex) != len(cst):
        problems.append("OceanTexture values differ from the header's ocean_texture")
    ver = int(re.search(r"#define OCEAN_ABI_VERSION (\d+)", hs).group(1))
    m = re.search(r"public const int AbiVersion = (\d+);", cs)
    if not m or int(m.group(1)) != ver:
        problems.append(f"OceanNative.AbiVersion != OCEAN_ABI_VERSION {ver}")
    awake = re.search(r"public void Awake\(\)\s*\{(.*?)\n        \}", facade, flags=re.S)
    if not awake or not re.search(r"ocean_abi_version\(\)\s*!=\s*OceanNative\.AbiVersion\)\s*\n?\s*throw", awake.group(1)):
        problems.append("WaterBodyNative.Awake does not refuse a library of another ABI version")
    return problems


def _texts():
    return open(HEADER).read(), open(NATIVE).read(), open(FACADE).read()


def test_csharp_binding_matches_header():
    h, cs, facade = _texts()
    assert len(header_prototypes(h)) >= 38
    assert check_binding(h, cs, facade) == []


MUTANTS = {
    "dropped_parameter": (NATIVE, "ocean_step(IntPtr ctx, float time)", "ocean_step(IntPtr ctx)"),
    "wrong_parameter_type": (NATIVE, "ocean_ifft2d(IntPtr ctx, int planeMask)", "ocean_ifft2d(IntPtr ctx, float planeMask)"),
    "size_as_int": (NATIVE, "ocean_read_height_async(IntPtr ctx, int tile, int cascade, IntPtr dst, UIntPtr bytes,",
                    "ocean_read_height_async(IntPtr ctx, int tile, int cascade, IntPtr dst, int bytes,"),
    "swapped_struct_fields": (NATIVE, "public float wavelength, cutoffLow, cutoffHigh, swell, fade;",
                              "public float wavelength, cutoffHigh, cutoffLow, swell, fade;"),
    "wrong_version": (NATIVE, "public const int AbiVersion = 4;", "public const int AbiVersion = 3;"),
    "missing_entry": (NATIVE, "public static extern OceanStatus ocean_set_readback_timing(IntPtr ctx, int enable);",
                      "public static extern OceanStatus ocean_set_readback_timer(IntPtr ctx, int enable);"),
    "flag_value": (NATIVE, "Mips = 0x8,", "Mips = 0x10,"),
    "awake_no_check": (FACADE, "if (OceanNative.ocean_abi_version() != OceanNative.AbiVersion)", "if (false)"),
}


@pytest.mark.parametrize("mutant", sorted(MUTANTS))
def test_checker_catches_broken_binding(mutant):
    path, old, new = MUTANTS[mutant]
    h, cs, facade = _texts()
    text = cs if path == NATIVE else facade
    assert old in text, f"mutant {mutant} no longer applies"
    text = text.replace(old, new)
    problems = check_binding(h, text, facade) if path == NATIVE else check_binding(h, cs, text)
    assert problems, f"mutant {mutant} survived"
