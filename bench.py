#!/usr/bin/env python3
"""Benchmark of the per-frame ocean path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg3|cfg1|cfg2|cfg4|cfg5]

cfg1 (BASELINE.json configs[0], 256^2 x 1 on the scalar CPU path, no GPU) prints its own line with
n_gpus 0: the C port timed as the labelled stand-in for the C# path (run_cfg1).

A "step" is one ocean frame: ocean_step(t) = evolve -> 2D IFFT of every plane
-> fill/foam for every (tile, cascade) unit the rank owns (WaterBody.cs:180-193
minus GenerateMips), inputs resident in HBM.  Multi-GPU: one process per GPU
(torchrun).  cfg2/cfg3 scale weakly (every rank runs its own ocean); cfg4 and
cfg5 split one job (ocean_hip.shard.plan_shard: tile blocks for cfg4; cascades,
then even / odd columns for cfg5 -- at 8 GPUs each rank owns one 4096^2 cascade's
even or odd columns, ocean_set_column_parity).  No data-path collective exists; gloo carries only the
start/stop barrier and the max-over-ranks of the elapsed time.  `value` =
ocean-frames of the configured job (4 x 1024^2 cascades for cfg3) completed per
second over all ranks.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ocean-simulation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before ocean_hip: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

import ocean_hip as oh  # noqa: E402
from ocean_hip.shard import plan_shard, reduce_timing, tile_seed  # noqa: E402

PREWARM_S = 0.5  # device clock ramp before the warm-up steps (see main)
HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md (chip-level parameters)
HBM_COPY_GBS = 6290.0  # the same guide's measured float4 copy rate; SURVEY.md 8d asks for both fractions

SCENE_PARAMS = dict(wind_speed=8.0, wind_dir_x=1.0, wind_dir_y=-1.0, gravity=9.81, fetch=50000.0, depth=2560.0)
SCENE_CASCADES = [  # Assets/Scenes/Waves.unity (+ unreferenced 4th cascade :1572-1576)
    dict(wavelength=1530.0, cutoff_low=1e-10, cutoff_high=1e12, swell=0.4, fade=0.1),
    dict(wavelength=1000.0, cutoff_low=1e-7, cutoff_high=1e7, swell=0.3, fade=0.2),
    dict(wavelength=201.0, cutoff_low=1e-5, cutoff_high=1e6, swell=0.1, fade=0.1),
    dict(wavelength=34.0, cutoff_low=0.001, cutoff_high=10.0, swell=0.4, fade=0.1),
]

# BASELINE.json configs (tiles are per job; sharded over ranks)
CONFIGS = {
    "cfg1": dict(n=256, cascades=1, tiles=1, disp_only=False, per_rank=True, cpu_only=True,
                 desc="1 x 256^2 cascade, JONSWAP/TMA spectrum + 2D IFFT on the scalar CPU path (no GPU)"),
    "cfg2": dict(n=512, cascades=1, tiles=1, disp_only=True, per_rank=True,
                 desc="1 x 512^2 cascade, displacement only"),
    "cfg3": dict(n=1024, cascades=4, tiles=1, disp_only=False, per_rank=True,
                 desc="4 x 1024^2 cascades, displacement + derivatives + Jacobian foam"),
    "cfg4": dict(n=512, cascades=4, tiles=256, disp_only=False, per_rank=False,
                 desc="256 tiles x 4 x 512^2 cascades, sharded over ranks"),
    "cfg5": dict(n=4096, cascades=4, tiles=1, disp_only=False, per_rank=False,
                 desc="4 x 4096^2 cascades, split over ranks (cascades, then even / odd columns)"),
}


def algorithmic_bytes(ctx):
    """Per-step algorithmic HBM bytes of the schedule the context runs, from the library
    (ocean_step_bytes): N = 1024 full outputs, pass A4: 8 (h0k) + 32
    (4 planes) and pass B: 32 (planes) + 4 + 4 (foam state) + 48 (DISP, DERIV, TURB) per texel."""
    a, b = ctx.step_bytes()
    tex = ctx.n * ctx.n * ctx.C * ctx.T
    # bytes a frame reads that the previous kernels wrote / read (h0k or h0, the P-plane
    # intermediate, the foam state): what the 256 MiB Infinity Cache can keep between frames
    # (pass A reads the h0 bytes and writes the intermediate: together a; the foam state is 4 B)
    resident = a + (4 * tex if ctx.planes == 4 else 0)
    return {"pass_a": a, "pass_b": b, "frame": a + b, "cache_resident": resident}


PROFILES = os.path.join(ROOT, "profiles")


def _norm(sym):
    return " ".join(sym.split()) if sym else sym


_IDENT = {}


def library_identity():
    """sha256 of the liboceanhip.so this process loaded and of the library's sources (tools/stamp.py)."""
    if not _IDENT:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import stamp as st
        _IDENT.update(lib=st.lib_sha(oh.LIB_PATH), src=st.src_sha())
    return _IDENT


def find_record(config, symbol, profiles_dir=PROFILES):
    """The committed rocprofv3 record of `config` that holds the kernel `symbol` (the exact demangled
    name of the kernel that ran, ocean_kernel_name): profiles/<tag>/ with stamp.json (tools/profile.sh +
    tools/pmc_summary.py), kernel_stats.csv and pmc_summary.json.  Among those, the one whose stamp
    matches the loaded library's sha256, else its sources' sha256, else the newest stamp (UTC) -- never
    a directory-name order.  Unstamped directories (before round 4) are not considered.  Returns
    {dir, avg_us, launches, traffic_bytes_per_launch, match, utc} or None."""
    import csv
    if not symbol or not os.path.isdir(profiles_dir):
        return None
    want, ident = _norm(symbol), library_identity()
    best, best_key = None, None
    for d in os.listdir(profiles_dir):
        sp = os.path.join(profiles_dir, d, "stamp.json")
        ks = os.path.join(profiles_dir, d, "kernel_stats.csv")
        if not (os.path.exists(sp) and os.path.exists(ks)):
            continue
        try:
            stamp = json.load(open(sp))
        except Exception:
            continue
        if stamp.get("config") != config:
            continue
        row = next((r for r in csv.DictReader(open(ks)) if _norm(r["Name"]) == want), None)
        if row is None:
            continue
        match = "lib" if stamp.get("lib_sha256") == ident["lib"] else (
            "src" if stamp.get("src_sha256") == ident["src"] else "none")
        key = ({"lib": 2, "src": 1, "none": 0}[match], stamp.get("utc", ""))
        if best_key is not None and key <= best_key:
            continue
        traffic = None
        pp = os.path.join(profiles_dir, d, "pmc_summary.json")
        if os.path.exists(pp):
            rec = next((v for k, v in json.load(open(pp)).get("kernels", {}).items() if _norm(k) == want), None)
            traffic = rec["hbm_bytes_per_launch"] if rec else None
        best_key = key
        best = {"dir": f"profiles/{d}", "avg_us": float(row["AverageNs"]) / 1e3, "launches": int(row["Calls"]),
                "traffic_bytes_per_launch": traffic, "match": match, "utc": stamp.get("utc"),
                "git_head": stamp.get("git_head")}
    return best


def entry_record(config, symbol, profiles_dir=PROFILES):
    """The record of one timed entry of a kernel kind (find_record per kernel, summed): one kernel, except
    the N >= 2048 column passes, where each (unit, band) entry launches C1 (k_col4s1) then C2 (k_col4s2,
    the symbol the library reports as the kind's last kernel).  None unless every kernel of the entry
    has a record, all in one directory."""
    syms = [symbol] if symbol else []
    if symbol and "k_col4s2<" in symbol:
        syms = [re.sub(r"k_col4s2<(\d+), \d+, ", r"k_col4s1<\1, ", symbol), symbol]
    recs = [find_record(config, sym, profiles_dir) for sym in syms]
    if not recs or not all(recs) or len({r["dir"] for r in recs}) != 1:
        return None
    record = dict(recs[-1])
    record["avg_us"] = sum(r["avg_us"] for r in recs)
    tb = [r["traffic_bytes_per_launch"] for r in recs]
    record["traffic_bytes_per_launch"] = sum(tb) if all(t is not None for t in tb) else None
    record["kernels"] = syms
    return record


def _ceiling_dirs(fname, profiles_dir):
    """Directories holding the micro-benchmark record `fname` (wrbench.txt, aqbench.txt, bqbench.txt)
    with a ceilings.json stamp (tools/stamp.py --ceilings), best first: records made by the current
    code of the tool before others, then the newest stamp (UTC).  Directory names play no part, so the
    quoted ceilings do not depend on the round."""
    if not os.path.isdir(profiles_dir):
        return []
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import stamp as st
    tool = st.CEILING_TOOLS[fname]
    tool_path = os.path.join(ROOT, "tools", tool)
    cur = st.code_sha(tool_path) if os.path.exists(tool_path) else None
    found = []
    for d in os.listdir(profiles_dir):
        sp = os.path.join(profiles_dir, d, "ceilings.json")
        if not (os.path.exists(os.path.join(profiles_dir, d, fname)) and os.path.exists(sp)):
            continue
        try:
            s = json.load(open(sp))
        except Exception:
            continue
        match = cur is not None and s.get("tool_code_sha256", {}).get(tool) == cur
        found.append(((match, s.get("utc", "")), d))
    return [d for _, d in sorted(found, reverse=True)]


def write_ceilings(profiles_dir=os.path.join(ROOT, "profiles")):
    """Measured store-bandwidth ceilings of this chip from the best stamped tools/wrbench.hip record
    (_ceiling_dirs): GB/s of nontemporal float4 stores over 192 MiB (pass B's texture bytes) and
    beyond the Infinity Cache (1 GiB).  None if no stamped record exists."""
    for d in _ceiling_dirs("wrbench.txt", profiles_dir):
        got = {}
        for line in open(os.path.join(profiles_dir, d, "wrbench.txt")):
            m = re.match(r"(write \w+ (?:192 MiB|1 GiB))\s+grid\s+\d+\s+[\d.]+ us\s+([\d.]+) GB/s", line)
            if m:
                got[m.group(1)] = float(m.group(2))
        if "write nt 192 MiB" in got:
            return {"nt_192MiB_GBs": got["write nt 192 MiB"], "nt_beyond_cache_GBs": got.get("write nt 1 GiB"),
                    "source": f"profiles/{d}/wrbench.txt"}
    return None


def shape_us(fname, label, profiles_dir=os.path.join(ROOT, "profiles")):
    """Microsecond time of the line starting with `label` in the best stamped <fname> record
    (_ceiling_dirs; tools/aqbench.hip, tools/bqbench.hip: a pass's memory shape run without its
    evolve / FFT work, 4 x 1024^2).  (us, source) or None."""
    for d in _ceiling_dirs(fname, profiles_dir):
        for line in open(os.path.join(profiles_dir, d, fname)):
            m = re.match(re.escape(label) + r"\s+([\d.]+) us", line)
            if m:
                return float(m.group(1)), f"profiles/{d}/{fname}"
    return None


def beyond_cache(steps=20):
    """The frame on a working set far beyond the 256 MiB Infinity Cache: cfg4's per-GPU shard at
    8 GPUs (32 tiles x 4 x 512^2, 128 units, ~1.2 GiB of per-frame data and a 1 GiB re-read set),
    so the frame's bytes are HBM bytes.  Returns frames' algorithmic bytes / time as a fraction
    of the HBM peak."""
    ctx = oh.OceanContext(512, 4, 32, 0)
    try:
        ctx.set_params(SCENE_PARAMS, SCENE_CASCADES)
        ctx.generate_noise_device(20251121)
        ctx.init_spectrum()
        for f in range(5):
            ctx.step(f / 60.0)
        ctx.synchronize()
        t0 = time.perf_counter()
        for f in range(steps):
            ctx.step((5 + f) / 60.0)
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / steps
        a, b = ctx.step_bytes()
        return {"workload": "32 tiles x 4 x 512^2 (cfg4 shard of one GPU at 8 GPUs), fused frame",
                "bytes_per_step": a + b, "ms_per_step": round(dt * 1e3, 4),
                "achieved_GBs": round((a + b) / dt / 1e9, 1),
                "frac": round((a + b) / dt / 1e9 / HBM_PEAK_GBS, 4)}
    finally:
        ctx.close()


def ifft_measure(ctx, reps, record_config):
    """The operator IFFT (ocean_ifft2d over the 4 planes, IFFT.InverseFastFourierTransform x 4) of a
    context: wall time (no events) and kernel time (HIP events attached to every launch) per call,
    algorithmic bytes 32 B per texel per plane (two passes x read + write), the symbols of the row
    and column kernels that ran, and the committed rocprofv3 / PMC records of exactly those symbols
    (find_record: the record of `record_config` stamped with this library).
    Every call transforms freshly evolved planes (ocean_evolve before it): the unnormalised inverse
    transform grows the data by ~N per call, to inf / NaN within a dozen calls, and constant or zero
    data runs at a higher clock (MI355X_MICROARCH.md).  Wall = (evolve + operator) - (evolve alone)."""
    n, units = ctx.n, ctx.C * ctx.T
    for k in range(5):  # first launches load the row/column code objects: keep them out of the timing
        ctx.evolve(0.1 * k)
        ctx.ifft2d(0b1111)
    ctx.synchronize()
    s0 = time.perf_counter()  # wall regions: no events
    for k in range(reps):
        ctx.evolve(0.5 + k / 60.0)
        ctx.ifft2d(0b1111)
    ctx.synchronize()
    s1 = time.perf_counter()
    for k in range(reps):
        ctx.evolve(0.5 + k / 60.0)
    ctx.synchronize()
    s2 = time.perf_counter()
    ctx.set_kernel_timing(True)  # kernel region: events around every launch (evolve is kind 2)
    ctx.kernel_stats(0), ctx.kernel_stats(1), ctx.kernel_stats(2)
    for k in range(reps):
        ctx.evolve(0.5 + k / 60.0)
        ctx.ifft2d(0b1111)
    r_ms, r_n = ctx.kernel_stats(0)
    c_ms, c_n = ctx.kernel_stats(1)
    ctx.kernel_stats(2)
    ctx.set_kernel_timing(False)
    syms = {"rows": ctx.kernel_name(0), "cols": ctx.kernel_name(1)}
    fft_bytes = 32 * n * n * 4 * units
    stage_us = 1e6 * ((s1 - s0) - (s2 - s1)) / reps
    kern_us = 1e3 * (r_ms + c_ms) / reps
    rp = {k: find_record(record_config, v) for k, v in syms.items()} if record_config else {}
    rocprof = traffic = None
    lr, lc = r_n / reps, c_n / reps  # launches per call: rows and columns may run per unit chunk (ocean_abi.cpp)
    if rp.get("rows") and rp.get("cols"):
        rus = rp["rows"]["avg_us"] * lr + rp["cols"]["avg_us"] * lc
        rocprof = {"source": rp["cols"]["dir"], "record_match": rp["cols"]["match"], "utc": rp["cols"]["utc"],
                   "rows_us": round(rp["rows"]["avg_us"], 2), "cols_us": round(rp["cols"]["avg_us"], 2),
                   "launches_per_call": [lr, lc], "achieved_GBs": round(fft_bytes / (rus * 1e-6) / 1e9, 1),
                   "frac": round(fft_bytes / (rus * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
        tr, tc = rp["rows"]["traffic_bytes_per_launch"], rp["cols"]["traffic_bytes_per_launch"]
        if tr and tc:
            traffic = {"rows_bytes_per_launch": tr, "cols_bytes_per_launch": tc,
                       "bytes_per_call": int(tr * lr + tc * lc), "algorithmic_bytes_per_call": fft_bytes,
                       "source": rp["cols"]["dir"]}
    return {"bytes": fft_bytes, "us_per_stage_wall": round(stage_us, 2), "us_per_stage_kernels": round(kern_us, 2),
            "row_launches": r_n // reps, "col_launches": c_n // reps,
            "rows_us": round(1e3 * r_ms / reps, 2), "cols_us": round(1e3 * c_ms / reps, 2),
            "rows_frac": round(fft_bytes / 2 / (1e3 * r_ms / reps * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "cols_frac": round(fft_bytes / 2 / (1e3 * c_ms / reps * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "achieved_GBs": round(fft_bytes / (kern_us * 1e-6) / 1e9, 1),
            "frac": round(fft_bytes / (kern_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "wall_frac": round(fft_bytes / (stage_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "wall_frac_of_measured_copy": round(fft_bytes / (stage_us * 1e-6) / 1e9 / HBM_COPY_GBS, 4),
            "symbols": syms, "rocprof": rocprof, "traffic": traffic}


def ifft_beyond_cache(reps=50):
    """The operator IFFT at N = 1024 on a plane set twice the 256 MiB Infinity Cache: 4 tiles x 4
    cascades x 4 planes = 512 MiB, so the operator's bytes cannot all be
    cache-resident between its launches."""
    ctx = oh.OceanContext(1024, 4, 4, oh.F_UNFUSED)
    try:
        ctx.set_params(SCENE_PARAMS, SCENE_CASCADES)
        ctx.generate_noise_device(20251121)
        ctx.init_spectrum()
        r = ifft_measure(ctx, reps, "ifft_bc")
        r["workload"] = "4 tiles x 4 cascades x 1024^2, 4 planes: 512 MiB of planes (2x the Infinity Cache)"
        r["data"] = "freshly evolved planes before every call (frame data)"
        return r
    finally:
        ctx.close()


def mip_record(profiles_dir=PROFILES):
    """The mip kernels' time per frame from the committed rocprofv3 record of the update loop (config
    "update_loop", tools/profile.sh running `bench.py --only-update-loop`): the k_mips_* kernels of the
    record chosen by find_record's rule (stamp matching the loaded library first), total duration per
    frame."""
    import re
    names = ("ocean::(anonymous namespace)::k_mips_block(ocean::DevView, int, int)",
             "ocean::(anonymous namespace)::k_mips_tail(ocean::DevView, int)")
    recs = {nm: find_record("update_loop", nm, profiles_dir) for nm in names}
    if any(r is None for r in recs.values()) or len({r["dir"] for r in recs.values()}) != 1:
        return None
    # ocean_step launches k_mips_block once per frame (both chains, every slice), then k_mips_tail when
    # the chain is deeper than one block's levels (csrc/mips.hip): frames = the block kernel's calls
    frames = recs[names[0]]["launches"]
    us = sum(r["avg_us"] * r["launches"] for r in recs.values()) / frames
    r0 = next(iter(recs.values()))
    return {"dir": r0["dir"], "match": r0["match"], "utc": r0["utc"], "us_per_frame": round(us, 2),
            "kernels": {re.search(r"k_\w+", nm).group(0): {"avg_us": round(r["avg_us"], 3), "launches": r["launches"]}
                        for nm, r in recs.items()}}


UPDATE_WARM_S = 0.5  # Update-loop warm-up, wall seconds (update_loop)


def numa_placement(device, host_ptrs):
    """NUMA nodes that set the readback link rate: the GPU's (sysfs, from its PCI address), the calling
    CPU's, and the node of the first page of each pinned host buffer (get_mempolicy(MPOL_F_NODE |
    MPOL_F_ADDR)).  A pinned ring on the far socket crosses the inter-socket link (tools/d2hbench.hip
    measures both placements); None where the system does not say."""
    import ctypes
    out = {"gpu_node": None, "cpu": None, "cpu_node": None, "pinned_page_nodes": []}
    try:
        pr = torch.cuda.get_device_properties(device)
        bus = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        out["gpu_pci"] = bus
        out["gpu_node"] = int(open(f"/sys/bus/pci/devices/{bus}/numa_node").read())
    except Exception:
        pass
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        cpu = libc.sched_getcpu()
        out["cpu"] = cpu
        for node in range(64):
            if os.path.exists(f"/sys/devices/system/node/node{node}/cpu{cpu}"):
                out["cpu_node"] = node
                break
        for p in host_ptrs:
            node = ctypes.c_int(-1)
            r = libc.syscall(ctypes.c_long(239), ctypes.byref(node), None, ctypes.c_ulong(0), ctypes.c_void_p(p),
                             ctypes.c_ulong(3))  # SYS_get_mempolicy (x86_64), MPOL_F_NODE | MPOL_F_ADDR
            out["pinned_page_nodes"].append(node.value if r == 0 else None)
    except Exception:
        pass
    return out


def _loop_mode(wb, steps, warmup, f0):
    """One readback mode of update_loop: warm-up by time, `steps` timed Update frames with no timing
    events anywhere (frames/s), then the same loop with readback timing on (the copies' own time,
    ocean_readback_copy_ms) and again with the frame's kernels timed (are the frames stretched by the
    copies beside them?).  Returns (record, next frame index)."""
    ctx = wb.ctx
    f = f0
    w0 = time.perf_counter()
    while f - f0 < max(warmup, 2 * len(wb._ring)) or time.perf_counter() - w0 < UPDATE_WARM_S:
        wb.Update(f / 60.0)
        f += 1
    wb.WaitForReadback()
    warm_frames, warm_s = f - f0, time.perf_counter() - w0
    t0 = time.perf_counter()
    for k in range(steps):
        wb.Update((f + k) / 60.0)
    wb.WaitForReadback()  # every requested readback has landed inside the timed region
    loop_s = (time.perf_counter() - t0) / steps
    f += steps
    wb.readback_copy_ms = []
    for k in range(steps):
        wb.Update((f + k) / 60.0)
    wb.WaitForReadback()
    f += steps
    copies = list(wb.readback_copy_ms)
    wb.readback_copy_ms = None
    ctx.set_kernel_timing(True)
    ctx.kernel_stats(0), ctx.kernel_stats(1), ctx.kernel_stats(2)
    for k in range(steps):
        wb.Update((f + k) / 60.0)
    wb.WaitForReadback()
    f += steps
    la, _ = ctx.kernel_stats(0)
    lb, _ = ctx.kernel_stats(1)
    lm, _ = ctx.kernel_stats(2)
    ctx.set_kernel_timing(False)
    slice_bytes = wb.texturesSize ** 2 * (4 if wb.readback == "height" else 16)
    copy_ms = float(np.median(copies)) if copies else None
    rec = {"readback": wb.readback, "frames_per_s": round(1.0 / loop_s, 2), "ms_per_frame": round(1e3 * loop_s, 4),
           "timed_frames": steps, "warmup": {"frames": warm_frames, "seconds": round(warm_s, 3)},
           "pcie_bytes_per_frame": slice_bytes, "pcie_GBs": round(slice_bytes / loop_s / 1e9, 2),
           "d2h": {"copies": len(copies), "median_ms": round(copy_ms, 4) if copy_ms else None,
                   "max_ms": round(max(copies), 4) if copies else None,
                   "GBs": round(slice_bytes / (copy_ms * 1e-3) / 1e9, 2) if copy_ms else None,
                   "how": "ocean_readback_copy_ms (readback timing on, a loop of its own): HIP events on the copy "
                          "stream around each device-to-host copy"},
           "kernel_us_in_loop": {"pass_a": round(1e3 * la / steps, 2), "pass_b": round(1e3 * lb / steps, 2),
                                 "other": round(1e3 * lm / steps, 2)}}
    return rec, f


def update_loop(steps=200, warmup=20):
    """The reference's per-frame loop at cfg3, as a Unity host over this library runs it
    (WaterBody.Update, WaterBody.cs:284-297): CalculateWavesTexturesAtTime with the mip chains of DERIV
    and TURB regenerated every frame (GenerateMips, :191-192; OCEAN_F_MIPS), then one asynchronous
    readback of displacement slice 0 per frame (AsyncGPUReadback.Request, :288) into the facade's
    pinned ring, polled, the landed slice kept in its pinned slot for GetWaterHeight -- ocean_hip.WaterBody.Update.
    Two readback modes, each its own facade and loop: "height" (the facade's default: DISP.y alone,
    ocean_read_height_async, 4 MiB per frame -- the reference's buoyancyData is private, WaterBody.cs:58,
    and GetWaterHeight reads only .g, :208) and "rgba" (the whole 16 MiB Color slice, as the reference
    requests it).  Reported beside `value` (the device frame without mips): each mode's
    frames/s with no timing events in its timed region, its PCIe bytes, the copies' own time (a second
    loop with readback timing on) and the frame's kernels inside the loop (a third, HIP events); the
    frame with mips alone, and the mip kernels' time.
    Warm-up is by time, not by count: the loop's first frames in a process run 3-13x slower
    (tools/update_ramp.py, docs/MEASUREMENTS.md section 8).  Every loop runs for >= UPDATE_WARM_S (and
    >= `warmup` frames) before its timed region."""
    out = {"workload": "cfg3 (4 x 1024^2) frame + GenerateMips of DERIV and TURB + AsyncGPUReadback of DISP "
                       "slice 0 every frame, ocean_hip.WaterBody.Update (WaterBody.cs:284-297)"}
    for mode in ("height", "rgba"):
        wb = oh.scene_water_body(n=1024, n_cascades=4, seed=20251121, readback=mode).Awake()
        ctx = wb.ctx
        try:
            if mode == "height":  # the frame with mips alone, once
                f = 0
                w0 = time.perf_counter()
                while f < warmup or time.perf_counter() - w0 < UPDATE_WARM_S:
                    ctx.step(f / 60.0)
                    f += 1
                    if f % 16 == 0:
                        ctx.synchronize()
                ctx.synchronize()
                t0 = time.perf_counter()
                for k in range(steps):
                    ctx.step((f + k) / 60.0)
                ctx.synchronize()
                step_s = (time.perf_counter() - t0) / steps
                ctx.set_kernel_timing(True)
                ctx.kernel_stats(0), ctx.kernel_stats(1), ctx.kernel_stats(2)
                for k in range(steps):
                    ctx.step((f + k) / 60.0)
                ka, _ = ctx.kernel_stats(0)
                kb, _ = ctx.kernel_stats(1)
                km, nm = ctx.kernel_stats(2)
                ctx.set_kernel_timing(False)
                out["step_with_mips"] = {"frames_per_s": round(1.0 / step_s, 2), "ms_per_frame": round(1e3 * step_s, 4),
                                         "kernel_us": {"pass_a": round(1e3 * ka / steps, 2), "pass_b": round(1e3 * kb / steps, 2),
                                                       "mips": round(1e3 * km / steps, 2)},
                                         "mip_launches_per_frame": nm / steps, "mips_symbol_last": ctx.kernel_name(2),
                                         "mips_rocprof": mip_record()}
                out["readback_ring_slots"] = wb._in_flight()
                out["numa"] = numa_placement(wb.device, [b.ptr.value for b in wb._ring])
            out[mode], _ = _loop_mode(wb, steps, warmup, 0)
        finally:
            wb.OnDisable()
    out["height_over_rgba"] = round(out["height"]["frames_per_s"] / out["rgba"]["frames_per_s"], 3)
    # top-level figures of the facades' default mode (height); "rgba" is the reference's own request
    out["frames_per_s"], out["ms_per_frame"] = out["height"]["frames_per_s"], out["height"]["ms_per_frame"]
    out["top_level_mode"] = "height"
    return out


def cpu_baseline(cfg, frames=3):
    """Scalar single-thread C port of the reference path (oracle/ocean_oracle.c), full frame
    (evolve + radix-2 IFFT of every plane + fill) on the host cores of this box."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    n, C = cfg["n"], cfg["cascades"]
    if n > 1024:  # bound the CPU sample (~10-30 s): time 1024^2 cascades and scale by texel count x log2N
        n_s = 1024
    else:
        n_s = n
    noise = O.generate_noise(n_s, 20251121)
    oc = O.OracleOcean(n_s, SCENE_PARAMS, SCENE_CASCADES[:C], noise, nplanes=2 if cfg["disp_only"] else 4)
    oc.step(0.0)  # warm-up
    ts = []
    for f in range(frames):
        t0 = time.perf_counter()
        oc.step((f + 1) / 60.0)
        ts.append(time.perf_counter() - t0)
    sec = float(np.median(ts))
    scale = (n * n * np.log2(n)) / (n_s * n_s * np.log2(n_s))
    sec *= scale
    per_tile = 1.0 / sec
    # secondary figure (Parallel.For over the host cores): the same frames on
    # the box's CPU share -- OMP_NUM_THREADS (16 per GPU on the GPU pool), else the cores
    threads = int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1))
    multi = None
    if threads > 1:
        O.set_threads(threads)
        try:
            oc.step(0.5)  # warm-up (thread pool start)
            tm = []
            for f in range(frames):
                t0 = time.perf_counter()
                oc.step((f + 1) / 30.0)
                tm.append(time.perf_counter() - t0)
        finally:
            O.set_threads(1)
        multi = {"value": 1.0 / (float(np.median(tm)) * scale), "cores": threads,
                 "sample": f"median of {frames} frames, OpenMP over the oracle's frame loops"}
    return {"value": per_tile, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"median of {frames} frames after 1 warm-up, 1 ocean of {C} x {n_s}^2 "
                      f"{'(scaled x%.2f to %d^2) ' % (scale, n) if scale != 1 else ''}"
                      f"on 1 host core; C port of the reference path (oracle/ocean_oracle.c), standing in for "
                      f"the C# scalar baseline of north_star (ocean-simulation_amd/csharp/CpuOcean.cs, "
                      f"compile-ready, same op order) because dotnet is absent on this image",
            "multicore": multi}


def run_cfg1(args):
    """BASELINE.json configs[0]: one 256^2 cascade through the reference path on the scalar CPU, no GPU
    (WaterBody.cs:171-193 on one core).  The path timed is the C port (oracle/ocean_oracle.c, the
    reference's four kernels in their op order, radix-2 schedule included), standing in, labelled, for
    the C# scalar re-implementation ocean-simulation_amd/csharp/CpuOcean.cs, which cannot run here: no
    dotnet on this image.  `value` = frames/s of CalculateWavesTexturesAtTime (evolve, 4 x 2D IFFT, fill
    and foam) over K timed frames after W warm-up frames; the initial spectrum (JONSWAP / TMA / spread,
    CalculateInitialSpectrumTextures) is timed once beside it.  n_gpus is 0."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    cfg = CONFIGS["cfg1"]
    n, C = cfg["n"], cfg["cascades"]
    O.set_threads(1)
    noise = O.generate_noise(n, 20251121)
    t0 = time.perf_counter()
    oc = O.OracleOcean(n, SCENE_PARAMS, SCENE_CASCADES[:C], noise)
    init_s = time.perf_counter() - t0
    for f in range(args.warmup):
        oc.step(f / 60.0)
    t0 = time.perf_counter()
    for f in range(args.steps):
        oc.step((args.warmup + f) / 60.0)
    elapsed = time.perf_counter() - t0
    return {
        "metric": f"ocean-surface frames/sec ({cfg['desc']})",
        "value": round(args.steps / elapsed, 2),
        "unit": "frames/s",
        "n_gpus": 0,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": None,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (scene parameters of Waves.unity, seeded noise 20251121)",
        "config": {"workload": f"cfg1: {cfg['desc']}", "n": n, "cascades": C, "tiles_per_gpu": None,
                   "parallelism": "one host core, no GPU"},
        "path": {"kind": "port", "cores": 1,
                 "what": "C port of the reference path (oracle/ocean_oracle.c, -O2 -ffp-contract=off), standing in "
                         "for the C# scalar path ocean-simulation_amd/csharp/CpuOcean.cs (same op order), which "
                         "cannot run here: no dotnet on this image",
                 "reference": "WaterBody.cs:171-193 (Awake's CalculateInitialSpectrumTextures, then "
                              "CalculateWavesTexturesAtTime per frame)"},
        "init_spectrum_ms": round(1e3 * init_s, 3),
        "roofline": None,  # no GPU kernel runs in this config
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--unfused", action="store_true", help="reference-shaped schedule (evolve, 4 x ifft2d, fill)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ifft-stage", action="store_true")
    ap.add_argument("--no-beyond-cache", action="store_true")
    ap.add_argument("--no-update-loop", action="store_true")
    ap.add_argument("--no-interleave", action="store_true",
                    help="cfg5 past one GPU per cascade: contiguous column bands instead of even / odd columns")
    ap.add_argument("--only-update-loop", action="store_true",
                    help="run update_loop alone and print its JSON (the rocprofv3 record of the mip kernels)")
    args = ap.parse_args()
    if CONFIGS[args.config].get("cpu_only"):
        print(json.dumps(run_cfg1(args)), flush=True)
        return
    if args.only_update_loop:
        print(json.dumps(update_loop(max(50, args.steps // 2), args.warmup)))
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # gloo prints its "[Gloo] Rank r is connected to ..." lines on stdout while the mesh
        # connects: send fd 1 to stderr meanwhile, so rank 0's stdout stays ONE JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    if args.gpus != world and not (world == 1 and args.gpus == 1):
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    cfg = CONFIGS[args.config]
    n = cfg["n"]
    if cfg["per_rank"]:
        # weak scaling: every rank runs its own ocean(s) (global tiles rank*T .. rank*T+T-1)
        tiles = cfg["tiles"]
        first = rank * tiles
        casc0, C, x0, nx = 0, cfg["cascades"], 0, n
        parity = -1
        job_oceans = tiles * world
    else:
        # strong scaling: the job's fixed oceans split over the ranks -- contiguous tile
        # blocks (cfg4), or one ocean's cascades and then column bands (cfg5 on 8 GPUs:
        # one cascade's even or odd columns per rank); no data exchange either way
        sh = plan_shard(cfg["tiles"], cfg["cascades"], n, world, rank, interleave=not args.no_interleave)
        first, tiles, casc0, C, x0, nx = sh.tile0, sh.tiles, sh.casc0, sh.cascades, sh.x0, sh.nx
        parity = sh.parity
        job_oceans = cfg["tiles"]
    flags = (oh.F_DISPLACEMENT_ONLY if cfg["disp_only"] else 0) | (oh.F_UNFUSED if args.unfused else 0)

    # one GPU per rank; more ranks than GPUs (a rehearsal of the N-rank path on a
    # smaller box) share devices round-robin
    device = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(device)
    ctx = oh.OceanContext(n, C, tiles, flags, device=device)
    ctx.set_params(SCENE_PARAMS, SCENE_CASCADES[casc0:casc0 + C])
    ctx.generate_noise(tile_seed(20251121, first))  # the reference shares one noise texture over cascades
    if parity >= 0:
        ctx.set_column_parity(parity)  # even / odd columns of the cascade (cfg5 on 8 GPUs)
    elif nx != n:
        ctx.set_column_band(x0, nx)
    ctx.init_spectrum()
    ctx.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    # device pre-warm: frames for >= PREWARM_S of wall time before the W warm-up steps, so a
    # short run (the driver's --steps 20 --warmup 5) does not time the clock ramp of an idle
    # GPU -- measured: pass A 39.0 us over 20 steps after 5 warm-ups against 33.2 us over 500
    # after 50 (profiles/r02d).  Untimed, outside the timed region, on the same inputs.
    prewarm_frames = 0
    p0 = time.perf_counter()
    while time.perf_counter() - p0 < PREWARM_S:
        for _ in range(8):
            ctx.step(-1.0 - prewarm_frames / 60.0)
            prewarm_frames += 1
        ctx.synchronize()
    prewarm_s = time.perf_counter() - p0
    # the prewarm frames advanced the foam state; the measured job starts from zero foam
    ctx.reset_foam()
    # warm-up
    for f in range(args.warmup):
        ctx.step(f / 60.0)
    ctx.synchronize()

    # timed region (`value`): K frames bracketed by barrier + device synchronize
    barrier()
    ctx.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in range(args.steps):
        ctx.step((args.warmup + f) / 60.0)
    ctx.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0

    # kernel region: the same K frames again with HIP events attached to every kernel
    # dispatch on the ctx stream (ocean_set_kernel_timing; hipExtLaunchKernel start/stop
    # events, so the durations are the kernels' own and agree with rocprofv3 --stats) ->
    # per-kernel average durations for the roofline.  Kept out of the timed region: the
    # event bookkeeping still lengthens a step by ~10 %.
    ctx.set_kernel_timing(True)
    ctx.kernel_stats(0), ctx.kernel_stats(1), ctx.kernel_stats(2)  # reset
    ctx.synchronize()
    t2 = time.perf_counter()
    for f in range(args.steps):
        ctx.step((args.warmup + args.steps + f) / 60.0)
    ctx.synchronize()
    t3 = time.perf_counter()
    elapsed_ev = t3 - t2
    ka_ms, ka_n = ctx.kernel_stats(0)
    kb_ms, kb_n = ctx.kernel_stats(1)
    ctx.set_kernel_timing(False)

    elapsed, _ = reduce_timing(elapsed, tiles, world)
    elapsed_ev, _ = reduce_timing(elapsed_ev, tiles, world)

    units = tiles * C
    B = algorithmic_bytes(ctx)
    # kernel time per step (a step may launch each pass once per unit chunk, ocean_abi.cpp
    # chunk_units); bytes per step / time per step = bytes per launch / time per launch
    a_us = 1e3 * ka_ms / args.steps
    b_us = 1e3 * kb_ms / args.steps
    dom, dom_us = ("pass_b", b_us) if b_us >= a_us else ("pass_a", a_us)
    # launches of the dominant kind per step (each pass runs once per unit chunk; at N >= 2048 the
    # column kind is C1 + C2 per (unit, band), so per-launch figures there mix the two kernels)
    launches_per_step = max(kb_n if dom == "pass_b" else ka_n, 1) / args.steps
    if args.unfused:
        dom = "ifft_cols" if dom == "pass_b" else "ifft_rows"
    dom_bytes = B["pass_b" if dom in ("pass_b", "ifft_cols") else "pass_a"]
    if args.unfused:  # unfused row/col launches move 16 B per texel per plane, all planes in one launch
        dom_bytes = n * n * units * 16 * (2 if cfg["disp_only"] else 4)
        if dom == "ifft_cols" and n >= 2048:  # four-step columns: C1 and C2 each read + write the planes
            dom_bytes *= 2
    achieved = dom_bytes / (dom_us * 1e-6) / 1e9 if dom_us > 0 else 0.0

    kernel_syms = {"pass_a": ctx.kernel_name(0), "pass_b": ctx.kernel_name(1)}
    dom_sym = kernel_syms["pass_b" if dom in ("pass_b", "ifft_cols") else "pass_a"]

    ifft_stage = None
    if not args.no_ifft_stage and not cfg["disp_only"]:
        # operator-level stage (IFFT.InverseFastFourierTransform x 4 planes), unfused kernels, on the
        # frame's own planes (ocean_evolve before every call): the fused frame never writes them, and
        # zero-filled planes run at a higher clock (MI355X_MICROARCH.md) -- rounds 1-2 timed zeros
        # rocprofv3 + PMC records of the operator's kernels (tools/profile.sh): config "ifft" for cfg3's
        # 4 x 1024^2 x 4 planes, "op4k" for the 4 x 4096^2 operator (the same launches per unit-plane
        # chunk as cfg5's)
        ifft_stage = ifft_measure(ctx, max(20, args.steps // 5), {"cfg3": "ifft", "cfg5": "op4k"}.get(args.config))
        ifft_stage["data"] = "freshly evolved planes before every call (frame data)"
        if rank == 0 and world == 1 and args.config == "cfg3" and not args.no_beyond_cache:
            ifft_stage["beyond_cache"] = ifft_beyond_cache()

    record = entry_record(args.config, dom_sym) if not args.unfused else None
    traffic = record["traffic_bytes_per_launch"] if record else None
    # the dominant kernel's store stream against the chip's measured store ceiling: pass B writes the
    # textures (16 B DISP [+ 32 B DERIV, TURB] [+ 16 B NORMAL]) and the 4-B foam state per texel
    writes = None
    if dom == "pass_b" and ctx.planes == 4:
        wb = ctx.n * ctx.n * ctx.C * ctx.T * (48 + 4)
        wc = write_ceilings()
        writes = {"bytes_per_launch": wb // max(1, round(launches_per_step)),
                  "achieved_GBs": round(wb / (dom_us * 1e-6) / 1e9, 1), "measured_ceiling": wc,
                  "frac_of_nt_ceiling": round(wb / (dom_us * 1e-6) / 1e9 / wc["nt_192MiB_GBs"], 4) if wc else None}
    # each pass against its own memory shape run without the evolve / FFT work (cfg3's shapes)
    shape = None
    if args.config == "cfg3" and not args.unfused and ctx.planes == 4 and n == 1024:
        sa = shape_us("aqbench.txt", "AQ rows (y, N - y), half lines")
        sb = shape_us("bqbench.txt", "texture layout, nt")
        shape = {k: {"kernel_us": round(u, 3), "shape_us": v[0], "frac_of_shape": round(v[0] / u, 4), "source": v[1]}
                 for k, u, v in (("pass_a", a_us, sa), ("pass_b", b_us, sb)) if v}
    cache = None
    if rank == 0 and world == 1 and args.config == "cfg3" and not args.no_beyond_cache:
        cache = {"resident_set_bytes": B["cache_resident"], "infinity_cache_bytes": 256 << 20,
                 "note": "the frame's re-read set (h0k + intermediate + foam state) fits the Infinity Cache, "
                         "so part of `achieved` is cache bandwidth; beyond_cache is the HBM-bound figure",
                 "beyond_cache": beyond_cache()}
    update = None
    if rank == 0 and world == 1 and args.config == "cfg3" and not args.unfused and not args.no_update_loop:
        update = update_loop(max(50, args.steps // 2), args.warmup)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg)

    if rank == 0:
        frames = args.steps * job_oceans  # ocean-frames (one frame of one ocean = all its cascades of N^2)
        value = frames / elapsed
        out = {
            "metric": "ocean-surface frames/sec (4x1024^2 cascades)" if args.config == "cfg3"
            else f"ocean-surface frames/sec ({cfg['desc']})",
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "prewarm": {"frames": prewarm_frames, "seconds": round(prewarm_s, 3)},
            "ms_per_step": round(1e3 * elapsed / args.steps, 5),
            "higher_is_better": True,
            "scaling": "weak" if cfg["per_rank"] else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (scene parameters of Waves.unity, seeded noise 20251121+tile)",
            "config": {"workload": f"{args.config}: {cfg['desc']}", "n": n, "cascades": cfg["cascades"],
                       "tiles_per_gpu": tiles, "tiles_total": job_oceans,
                       "rank0_shard": {"cascades": [casc0, casc0 + C],
                                       "columns": f"x = 2m + {parity}" if parity >= 0 else [x0, x0 + nx]},
                       "schedule": "unfused" if args.unfused else "fused (pass A + pass B)",
                       "parallelism": f"{'independent oceans' if cfg['per_rank'] else 'one job split'} "
                                      f"over {world} GPU(s), no collective"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "measured_copy_GBs": HBM_COPY_GBS, "frac_of_measured_copy": round(achieved / HBM_COPY_GBS, 4),
                         "traffic": traffic,  # HBM bytes per launch (PMC), like `achieved`
                         "traffic_per_step": int(traffic * launches_per_step) if traffic else None,
                         "traffic_source": record["dir"] if record else None,
                         "record": ({k: record[k] for k in ("dir", "match", "utc", "git_head", "avg_us", "kernels")}
                                    if record else None),  # avg_us and traffic: per timed entry (all its kernels)
                         "rocprof_frac": (round(dom_bytes / launches_per_step / (record["avg_us"] * 1e-6) / 1e9
                                                / HBM_PEAK_GBS, 4) if record else None),
                         "kernel_symbol": dom_sym,
                         "algorithmic_bytes_per_launch": int(dom_bytes / launches_per_step),
                         "algorithmic_bytes_per_step": dom_bytes, "kernel_us_per_step": round(dom_us, 3),
                         "launches_per_step": round(launches_per_step, 2),
                         "writes": writes, "memory_shape": shape},
            "kernels_us": {"pass_a" if not args.unfused else "rows": round(a_us, 3),
                           "pass_b" if not args.unfused else "cols": round(b_us, 3)},
            "frame": {"algorithmic_bytes_per_gpu": B["frame"],
                      "achieved_GBs_per_gpu": round(B["frame"] / (elapsed / args.steps) / 1e9, 1),
                      "frac_per_gpu": round(B["frame"] / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                      "frac_of_measured_copy_per_gpu": round(B["frame"] / (elapsed / args.steps) / 1e9 / HBM_COPY_GBS, 4),
                      "ms_per_step_with_kernel_events": round(1e3 * elapsed_ev / args.steps, 5)},
            "ifft_stage": ifft_stage,
            "cache": cache,
            "update_loop": update,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
