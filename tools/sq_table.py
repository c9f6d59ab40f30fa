#!/usr/bin/env python3
"""Per-launch medians of the SQ counter groups written by tools/pmc_sq.sh, for one kernel-name substring."""
import csv, glob, os, statistics, sys
pat = sys.argv[1] if len(sys.argv) > 1 else "k_pass_a3"
for d in sorted(glob.glob("gpurun_out/sq_*")):
    vals = {}
    for f in glob.glob(os.path.join(d, "g*", "run_counter_collection.csv")):
        per = {}
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            per.setdefault((r["Counter_Name"], r["Dispatch_Id"]), 0.0)
            per[(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
        by = {}
        for (c, _), v in per.items():
            by.setdefault(c, []).append(v)
        for c, l in by.items():
            vals[c] = statistics.median(l)
    cfg = open(os.path.join(d, "cfg")).read().strip()
    wc = vals.get("SQ_WAVE_CYCLES", 1)
    print(f"== {cfg}")
    print("  " + "  ".join(f"{k[3:]}={v/1e6:.2f}M" for k, v in sorted(vals.items())))
    print(f"  WAIT_ANY {vals.get('SQ_WAIT_ANY',0)/wc:.2f} WAIT_INST {vals.get('SQ_WAIT_INST_ANY',0)/wc:.2f} "
          f"ACTIVE {vals.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} VALU-active {vals.get('SQ_ACTIVE_INST_VALU',0)/wc:.2f} "
          f"LDS-wait {vals.get('SQ_WAIT_INST_LDS',0)/wc:.2f}")
