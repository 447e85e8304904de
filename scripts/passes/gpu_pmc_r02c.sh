#!/bin/bash
# PMC passes over make_shares_vec (fused MT19937 draw + split, 2^24, 3-of-5):
# FETCH_SIZE, WRITE_SIZE (separate passes, MI355X_MICROARCH.md), then SQ LDS/VALU counters.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out/pmc_r02c"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/q1 -o run --output-format csv -- python3 "$R/scripts/prof_fused.py" > "$O/q1.log" 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/q2 -o run --output-format csv -- python3 "$R/scripts/prof_fused.py" > "$O/q2.log" 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS --kernel-trace -d /tmp/q3 -o run --output-format csv -- python3 "$R/scripts/prof_fused.py" > "$O/q3.log" 2>&1 \
&& for d in q1 q2 q3; do find /tmp/$d -name "*counter_collection.csv" -exec cp {} "$O/$d.csv" \; ; done \
&& echo "== pmc done"
