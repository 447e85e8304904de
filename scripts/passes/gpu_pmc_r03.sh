#!/bin/bash
# SQ counter passes (one rocprofv3 run per counter group, --kernel-trace only)
# over the kernels named in $KINDS (scripts/prof_kernels_r03.py: aes, prng).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out/${TAG:-pmc_r03}"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
rc=0
for k in ${KINDS:-aes prng}; do
  for p in 1 2; do
    [ $rc = 0 ] || break
    eval "C=\$P$p"
    echo "== $k pass $p"
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d /tmp/pmc_${k}_$p -o run --output-format csv -- python3 "$R/scripts/prof_kernels_r03.py" $k > "$O/${k}_$p.log" 2>&1 || rc=$?
    find /tmp/pmc_${k}_$p -name "*counter_collection.csv" -exec cp {} "$O/${k}_$p.csv" \;
  done
done
echo "== pmc rc $rc"
exit $rc
