#!/bin/bash
# Round-5 pass z: SQ counters of the MT jump level (make_shares_vec 2^24 back
# to back), two --pmc runs (kernel trace only), for where its waves wait.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05z}
mkdir -p $O
export TMPDIR=/tmp
rc=0
cd /tmp
echo "== p1" && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE --kernel-trace -d /tmp/z1 -o run --output-format csv -- python3 "$R/scripts/msv_loop_gaps.py" 24 > "$R/$O/p1.log" 2>&1 || rc=$?
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 "$R/$O/p1.log"; exit $rc; }
echo "== p2" && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d /tmp/z2 -o run --output-format csv -- python3 "$R/scripts/msv_loop_gaps.py" 24 > "$R/$O/p2.log" 2>&1 || rc=$?
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 "$R/$O/p2.log"; exit $rc; }
cd "$R"
find /tmp/z1 -name "*counter_collection.csv" -exec cp {} $O/p1_counters.csv \;
find /tmp/z2 -name "*counter_collection.csv" -exec cp {} $O/p2_counters.csv \;
ls -la $O
echo "== rc $rc"
exit $rc
