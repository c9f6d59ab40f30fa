#!/usr/bin/env python3
"""Summarise a tools/pmc_sq_cmd.sh run into profiles/<tag>/sq_summary.json: per kernel (exact demangled
symbol) the per-dispatch median of every SQ counter, the kernel record of the trace pass (VGPRs, LDS,
average duration) and the derived shares of SQ_WAVE_CYCLES (MI355X_MICROARCH.md: WAIT_ANY = parked on
s_waitcnt / barrier, WAIT_INST_ANY = issue stall, ACTIVE_INST_ANY = issuing; the three are disjoint and
sum to about WAVE_CYCLES; cycles are quad-cycles).
    python tools/sq_summary.py gpurun_out/sq_<x> profiles/<tag> [--match substr ...] [--label text]"""
import argparse
import csv
import glob
import json
import os
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("dst")
ap.add_argument("--match", nargs="*", default=["k_pass", "k_rows2", "k_cols2", "k_opc", "k_col4"])
ap.add_argument("--label", default="")
a = ap.parse_args()
os.makedirs(a.dst, exist_ok=True)
per = {}
for f in glob.glob(os.path.join(a.src, "g*", "run_counter_collection.csv")):
    acc = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not any(m in k for m in a.match):
            continue
        key = (k, r["Counter_Name"], r["Dispatch_Id"])
        acc[key] = acc.get(key, 0.0) + float(r["Counter_Value"])
    for (k, c, _), v in acc.items():
        per.setdefault(k, {}).setdefault(c, []).append(v)
trace = {}
tf = os.path.join(a.src, "trace", "run_kernel_trace.csv")
if os.path.exists(tf):
    for r in csv.DictReader(open(tf)):
        k = r["Kernel_Name"]
        if k in per:
            t = trace.setdefault(k, {"durations": []})
            t["durations"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            for col in ("Arch_VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Workgroup_Size",
                        "Grid_Size", "Scratch_Size"):
                if col in r:
                    t[col] = r[col]
out = {"label": a.label, "source": a.src, "kernels": {}}
for k, cs in per.items():
    med = {c: statistics.median(v) for c, v in cs.items()}
    wc = med.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    rec = {"counters_median_per_dispatch": med, "dispatches": max(len(v) for v in cs.values()),
           "share_of_wave_cycles": {n: round(med[c] / wc, 4) for n, c in (
               ("wait_any", "SQ_WAIT_ANY"), ("wait_inst_any", "SQ_WAIT_INST_ANY"), ("active_inst_any", "SQ_ACTIVE_INST_ANY"),
               ("active_valu", "SQ_ACTIVE_INST_VALU"), ("active_lds", "SQ_ACTIVE_INST_LDS"),
               ("wait_inst_lds", "SQ_WAIT_INST_LDS")) if c in med}}
    if k in trace:
        t = dict(trace[k])
        d = t.pop("durations")
        t["avg_duration_ns"] = statistics.mean(d)
        rec["trace"] = t
    out["kernels"][k] = rec
json.dump(out, open(os.path.join(a.dst, "sq_summary.json"), "w"), indent=1)
for k, r in out["kernels"].items():
    print(k[:90], r["share_of_wave_cycles"], r.get("trace", {}).get("Arch_VGPR_Count"))
