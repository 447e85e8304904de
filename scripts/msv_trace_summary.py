#!/usr/bin/env python3
"""One make_shares_vec call's GPU timeline from a rocprofv3 kernel trace (+
memory-copy trace): the ops of the last call (the stretch after the last
jump-level launch's preceding gap > 200 us), with start offsets, durations
and the gaps between them.  usage: msv_trace_summary.py <dir with csvs> [calls to keep, default 3]"""
import csv
import glob
import json
import sys

d = sys.argv[1]
ops = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")))
ops.sort()
# calls: split where the gap to the previous op exceeds 200 us
calls, cur = [], []
for o in ops:
    if cur and o[0] - cur[-1][1] > 200_000:
        calls.append(cur)
        cur = []
    cur.append(o)
calls.append(cur)
out = []
keep = int(sys.argv[2]) if len(sys.argv) > 2 else 3
for c in calls[-keep:]:
    t0 = c[0][0]
    rows, prev = [], None
    for s, e, n in c:
        rows.append({"op": n, "start_us": (s - t0) / 1e3, "dur_us": (e - s) / 1e3,
                     "gap_us": None if prev is None else (s - prev) / 1e3})
        prev = e
    out.append({"span_us": (c[-1][1] - t0) / 1e3, "ops": rows})
print(json.dumps(out, indent=1))
