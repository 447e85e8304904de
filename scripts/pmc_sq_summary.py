#!/usr/bin/env python3
"""Per-kernel SQ counter summary of rocprofv3 --pmc counter_collection.csv
files (summed over dispatches; per-wave and per-dispatch averages).
    python scripts/pmc_sq_summary.py DIR [PREFIX ...]
"""
import collections
import csv
import glob
import json
import os
import sys


def load(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r.get("Kernel_Name", "")
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((p, r.get("Dispatch_Id", "")))
    return agg, disp


def main():
    d = sys.argv[1]
    prefixes = sys.argv[2:] or sorted({os.path.basename(p).rsplit("_", 1)[0] for p in glob.glob(os.path.join(d, "*.csv"))})
    out = {}
    for pre in prefixes:
        agg, disp = load(sorted(glob.glob(os.path.join(d, f"{pre}_*.csv"))))
        for k, v in agg.items():
            nd = max(1, len(disp[k]) // 2)
            w = v.get("SQ_WAVES", 0) or 1
            row = {"dispatches_per_pass": nd, **{c: x / nd for c, x in sorted(v.items())}}
            cyc = v.get("SQ_WAVE_CYCLES", 0)
            if cyc:
                for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                          "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU"):
                    if c in v:
                        row[c + "_frac_of_wave_cycles"] = v[c] / cyc
            if "SQ_INSTS_VALU" in v and w:
                row["valu_insts_per_wave"] = v["SQ_INSTS_VALU"] / w
            out[f"{pre}: {k[:90]}"] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
