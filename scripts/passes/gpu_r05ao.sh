#!/bin/bash
# Round-5 pass ao: SQ counters of the kept AES envelope kernels (encrypt to
# hex, one-pass decrypt) from scripts/aes_enc_time.py, two --pmc runs (kernel
# trace only).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05ao}
mkdir -p $O
export TMPDIR=/tmp
rc=0
cd /tmp
echo "== p1" && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE --kernel-trace -d /tmp/a1 -o run --output-format csv -- python3 "$R/scripts/aes_enc_time.py" > "$R/$O/p1.log" 2>&1 || rc=$?
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 "$R/$O/p1.log"; exit $rc; }
echo "== p2" && timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d /tmp/a2 -o run --output-format csv -- python3 "$R/scripts/aes_enc_time.py" > "$R/$O/p2.log" 2>&1 || rc=$?
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 "$R/$O/p2.log"; exit $rc; }
cd "$R"
find /tmp/a1 -name "*counter_collection.csv" -exec cp {} $O/p1_counters.csv \;
find /tmp/a2 -name "*counter_collection.csv" -exec cp {} $O/p2_counters.csv \;
ls -la $O
echo "== rc $rc"
exit $rc
