#!/bin/bash
# SQ counters of the fused draw + split kernel (two passes, kernel-trace only).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/pmc_fused"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d /tmp/pf1 -o run --output-format csv -- python3 "$R/scripts/prof_fused.py" > "$R/gpurun_out/pmc_fused/p1.log" 2>&1 \
&& timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM --kernel-trace -d /tmp/pf2 -o run --output-format csv -- python3 "$R/scripts/prof_fused.py" > "$R/gpurun_out/pmc_fused/p2.log" 2>&1 \
&& for d in pf1 pf2; do find /tmp/$d -name "*counter_collection.csv" -exec cp {} "$R/gpurun_out/pmc_fused/$d.csv" \; ; done \
&& echo "== pmc fused done"
