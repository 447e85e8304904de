#!/usr/bin/env python3
"""usage: mt_gen_probe_summary.py <rocprof dir> <mt_gen_probe.py JSON output>
Median mt_gen_kernel<3, ...> and mt_jump_kernel durations per (block, probe)."""
import csv
import glob
import json
import statistics
import sys

d, order = sys.argv[1], json.load(open(sys.argv[2]))["order"]
gen, jumps = [], []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "mt_gen_kernel<3" in n or "mt_gen_pc_kernel<3" in n:
            gen.append((int(r["Start_Timestamp"]), dur))
        elif "mt_jump_kernel" in n:
            jumps.append((int(r["Start_Timestamp"]), dur))
gen.sort()
out, i = [], 0
for o in order:
    ds = [g[1] for g in gen[i:i + o["calls"]]]
    i += o["calls"]
    out.append({**o, "gen_us_median": statistics.median(ds) if ds else None, "gen_us": ds})
print(json.dumps({"rows": out, "jump_us_median": statistics.median(j[1] for j in jumps) if jumps else None}, indent=1))
