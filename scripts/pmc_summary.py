#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into profiles/pmc_traffic.json.

Corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE
and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a
coalesced streaming read (TCC_EA0_RDREQ x 64 B for 128-B requests), so read
bytes = 2 x FETCH_SIZE x 1024 (cross-checked with TCC_EA0_RDREQ x 128 B);
WRITE_SIZE x 1024 is exact for streaming stores.

usage: pmc_summary.py <dir with pmc_fetch.csv pmc_write.csv pmc_req.csv> <out.json> [log2n] [source note]
"""
import csv
import json
import statistics
import sys
from collections import defaultdict

d, out = sys.argv[1], sys.argv[2]
N = 1 << int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 24
vals = defaultdict(lambda: defaultdict(list))
for name in ("pmc_fetch", "pmc_write", "pmc_req"):
    with open(f"{d}/{name}.csv") as f:
        for row in csv.DictReader(f):
            kn = row["Kernel_Name"]
            k = ("split" if "split_kernel" in kn else
                 "reconstruct" if "reconstruct_kernel" in kn else
                 "fused_draw_split" if ("mt_gen_kernel<3" in kn or "mt_gen_pc_kernel<3" in kn) else
                 "mask_accumulate" if "bounded_acc_kernel" in kn else None)
            if k:
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
alg = {"split": N * (8 + 2 * 66 + 5 * 66), "reconstruct": N * (3 * 66 + 8),
       "fused_draw_split": N * (8 + 5 * 66), "mask_accumulate": N * 16}
alg_rw = {"split": (N * (8 + 2 * 66), N * 5 * 66), "reconstruct": (N * 3 * 66, N * 8),
          "fused_draw_split": (N * 8, N * 5 * 66), "mask_accumulate": (N * 8, N * 8)}
res = {"source": sys.argv[4] if len(sys.argv) > 4 else f"rocprofv3 --pmc passes summarised from {d}", "N": N, "workload": "3-of-5 split / reconstruct xs=1,3,5 -> int64, 2^24 elements; fused MT draw + split "
                     "(make_shares_vec); mask accumulate (10 generators, float64 base)", "kernels": {}}
for k, c in vals.items():
    if not c.get("FETCH_SIZE") or not c.get("WRITE_SIZE") or not c.get("TCC_EA0_RDREQ_sum"):
        continue
    fetch = statistics.median(c["FETCH_SIZE"]) * 1024
    write = statistics.median(c["WRITE_SIZE"]) * 1024
    rdreq = statistics.median(c["TCC_EA0_RDREQ_sum"])
    wrreq = statistics.median(c["TCC_EA0_WRREQ_sum"])
    read = 2 * fetch
    res["kernels"][k] = {
        "launches": len(c["FETCH_SIZE"]), "FETCH_SIZE_bytes_raw": fetch, "read_bytes": read,
        "read_bytes_from_RDREQx128": rdreq * 128, "write_bytes": write, "TCC_EA0_WRREQ_sum": wrreq,
        "hbm_bytes_per_launch": read + write, "algorithmic_bytes_per_launch": alg[k],
        "algorithmic_read_write": alg_rw[k], "traffic_over_algorithmic": (read + write) / alg[k]}
res["split_bytes_per_launch"] = res["kernels"]["split"]["hbm_bytes_per_launch"]
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
