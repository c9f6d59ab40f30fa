#!/usr/bin/env python3
"""Static instruction mix of one kernel of a HIP source, by class, from the gfx950 device assembly:
    python tools/valu_breakdown.py csrc/fftq.hip 'k_pass_aq<1024, false, 0, true' [out.json] [hipcc flags...]
The kernel is matched as a substring of its demangled name.  The report is the whole kernel body by
instruction class, with the Payne-Hanek range reduction of sincosf (the blocks that multiply by the 2/pi
bits) counted separately as cold: |omega t| < 2^17 never reaches it."""
import collections
import json
import re
import subprocess
import sys

src, want = sys.argv[1], sys.argv[2]
out_json = sys.argv[3] if len(sys.argv) > 3 and not sys.argv[3].startswith("-") else None
extra = [a for a in sys.argv[3:] if a.startswith("-")]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "-fno-slp-vectorize", "-I../include", "--cuda-device-only", "-S", src, "-o", "/tmp/_vb.s"] + extra
subprocess.run(cmd, check=True, cwd="ocean-simulation_amd")
asm = open("/tmp/_vb.s").read().splitlines()

# find the kernel whose demangled name contains `want`
starts = [(i, re.match(r"^(_Z\S+):", l).group(1)) for i, l in enumerate(asm) if re.match(r"^_Z\S+:", l)]
names = subprocess.run(["c++filt"], input="\n".join(n for _, n in starts), capture_output=True, text=True).stdout.split("\n")
hit = [(i, n, d) for (i, n), d in zip(starts, names) if want in d]
if not hit:
    sys.exit(f"no kernel matching {want!r}")
i0, mangled, dem = hit[0]
body = []
for l in asm[i0 + 1:]:
    if l.startswith(".Lfunc_end") or l.startswith("\t.size") or re.match(r"^_Z\S+:", l):
        break
    body.append(l)

# basic blocks
blocks, cur = [], ("entry", [])
for l in body:
    m = re.match(r"^(\.LBB\S+):", l) or re.match(r"^; (%bb\.\d+):", l)
    if m:
        blocks.append(cur)
        cur = (m.group(1), [])
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    cur[1].append(t)
blocks.append(cur)


def cls(op):
    if op.startswith("v_"):
        if "cndmask" in op:
            return "valu_select"
        if op.startswith(("v_mov", "v_readfirstlane", "v_readlane", "v_writelane", "v_accvgpr")):
            return "valu_move"
        if op.startswith("v_pk_"):
            return "valu_packed"
        if re.match(r"v_(add|sub|subrev)_f32", op):
            return "valu_fadd"
        if re.match(r"v_mul_f32", op):
            return "valu_fmul"
        if re.match(r"v_(fma|fmac|mac|mad)_f32", op):
            return "valu_ffma"
        if re.match(r"v_(sin|cos|rcp|rsq|sqrt|exp|log|fract|frexp|ldexp|div)", op):
            return "valu_transcendental"
        if re.match(r"v_(cmp|cmpx)", op):
            return "valu_compare"
        if re.match(r"v_(cvt|rndne|trunc|floor|ceil)", op):
            return "valu_convert"
        return "valu_int_addr"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu_branch_wait"
    return "other"


# Payne-Hanek range reduction of sinf / cosf (|x| >= 2^17 after the fast Cody-Waite path): the block that
# multiplies the mantissa by the 2/pi bits (v_mad_u64_u32 chain) and shifts them into place (v_alignbit)
def cold_block(ins):
    return sum(t.startswith("v_mad_u64_u32") for t in ins) >= 4 and any(t.startswith("v_alignbit") for t in ins)


per = collections.Counter()
cold = collections.Counter()
for name, ins in blocks:
    is_cold = cold_block(ins)
    for t in ins:
        op = t.split()[0]
        (cold if is_cold else per)[cls(op)] += 1
valu = {k: v for k, v in per.items() if k.startswith("valu")}
res = {"kernel": dem.strip(), "source": src, "flags": extra,
       "static_counts": dict(sorted(per.items())), "static_valu_total": sum(valu.values()),
       "cold_blocks_counts": dict(sorted(cold.items())),
       "note": "static counts over the kernel body; the Payne-Hanek blocks of sincosf (never reached at |omega t| < 2^17) counted as cold"}
print(json.dumps(res, indent=1))
if out_json:
    json.dump(res, open(out_json, "w"), indent=1)
