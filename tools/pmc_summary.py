#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>/:
kernel_stats.csv (rocprofv3 --kernel-trace --stats) and pmc_summary.json with the
per-launch HBM traffic of each kernel = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes).
gfx950 reports half the bytes of wide coalesced streaming reads in FETCH_SIZE
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section), hence the factor 2; the
Infinity Cache hits are included in FETCH_SIZE as well.

    python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag> [--config cfg3]

The record is stamped (profiles/<tag>/stamp.json): the box-side stamp of tools/profile.sh (config,
library and source sha256 of what ran, UTC time) plus the git HEAD of this tree and whether the
library's sources differed from it.  The config defaults to the stamp's.
"""
import argparse
import csv
import json
import os
import shutil
import statistics
import subprocess

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("dst")
ap.add_argument("--config", default=None)
a = ap.parse_args()
os.makedirs(a.dst, exist_ok=True)
stamp_path = os.path.join(a.src, "stamp.json")
stamp = json.load(open(stamp_path)) if os.path.exists(stamp_path) else {}
a.config = a.config or stamp.get("config") or "cfg3"
stamp["config"] = a.config
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
try:
    stamp["git_head"] = subprocess.check_output(["git", "-C", root, "rev-parse", "HEAD"], text=True).strip()
    dirty = subprocess.check_output(["git", "-C", root, "status", "--porcelain", "--", "ocean-simulation_amd/csrc",
                                     "include"], text=True).strip()
    stamp["src_dirty_vs_head"] = bool(dirty)
except Exception:
    stamp["git_head"] = None
json.dump(stamp, open(os.path.join(a.dst, "stamp.json"), "w"), indent=1)
shutil.copy(os.path.join(a.src, "trace", "run_kernel_stats.csv"), os.path.join(a.dst, "kernel_stats.csv"))
agg = {}
for kind in ("fetch", "write"):
    for r in csv.DictReader(open(os.path.join(a.src, kind, "run_counter_collection.csv"))):
        agg.setdefault(r["Kernel_Name"], {}).setdefault(kind, []).append(float(r["Counter_Value"]))
dur = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open(os.path.join(a.src, "trace", "run_kernel_stats.csv")))}
out = {"config": a.config, "stamp": stamp, "counters": "FETCH_SIZE, WRITE_SIZE (KB, separate --pmc passes)",
       "formula": "hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024", "kernels": {}}
for k, v in agg.items():
    f = statistics.median(v.get("fetch", [0.0]))
    w = statistics.median(v.get("write", [0.0]))
    out["kernels"][k] = {"launches": len(v.get("fetch", [])), "fetch_kb_median": f, "write_kb_median": w,
                         "hbm_bytes_per_launch": int((2 * f + w) * 1024), "avg_duration_ns": dur.get(k)}
json.dump(out, open(os.path.join(a.dst, "pmc_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1)[:2000])
