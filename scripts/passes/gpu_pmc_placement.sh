#!/bin/bash
# One rocprofv3 --pmc pass per counter group (kernel-trace only), placement workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"
mkdir -p gpurun_out/pmc_place
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum" \
           "TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" \
           "TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_TAG_STALL_sum" \
           "TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_STALL_MULTI_MISS_sum" \
           "TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum" \
           "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace -d /tmp/pp$i -o run --output-format csv -- python3 "$R/scripts/pmc_placement.py" > "$R/gpurun_out/pmc_place/p$i.log" 2>&1 || exit $?
  find /tmp/pp$i -name "*counter_collection.csv" -exec cp {} "$R/gpurun_out/pmc_place/p${i}_cc.csv" \;
  find /tmp/pp$i -name "*kernel_trace.csv" -exec cp {} "$R/gpurun_out/pmc_place/p${i}_kt.csv" \;
done
echo "== pmc placement done"
