#!/usr/bin/env python3
"""Join each placement PMC pass's counters with its kernel-trace durations (per dispatch)."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_place"
for cc in sorted(glob.glob(os.path.join(d, "p*_cc.csv"))):
    kt = cc.replace("_cc.csv", "_kt.csv")
    vals = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(cc)):
        if "split_kernel" not in r["Kernel_Name"]:
            continue
        vals[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    dur = {}
    if os.path.exists(kt):
        for r in csv.DictReader(open(kt)):
            if "split_kernel" in r["Kernel_Name"]:
                dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print("==", os.path.basename(cc))
    for disp in sorted(vals):
        print(f"  {disp:4d} {dur.get(disp, float('nan')):7.3f} ms  " +
              "  ".join(f"{k}={v:.4g}" for k, v in sorted(vals[disp].items())))
