#!/bin/bash
# Round-6 pass d: the envelope decrypt kernel without loop spills and with the
# next unit's text in flight across the AES — alternating-process A/B against
# HEAD's library (scripts/aes_enc_time.py), the AES GPU tests, then the SQ
# counters of the new kernels (two --pmc runs, kernel trace only).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06d}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rc=0
for round in 1 2 3; do
  for lib in ab/libdn_shamir_HEAD.so libdn_shamir.so; do
    DN_SHAMIR_LIB=delta-node_amd/lib/$lib timeout -k 10 120 python scripts/aes_enc_time.py >> $O/aes_ab.jsonl 2>> $O/aes_ab.err || { rc=$?; echo "== $lib rc $rc"; tail -3 $O/aes_ab.err; exit $rc; }
  done
done
cut -c1-260 $O/aes_ab.jsonl
echo "== pytest aes" && timeout -k 10 600 python -u -m pytest tests/test_gpu_aes.py tests/test_gpu_codec.py -x -q --timeout 300 --timeout-method thread > $O/pytest_aes.log 2>&1 || rc=$?
tail -2 $O/pytest_aes.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest_aes.log | head -5; exit $rc; }
cd /tmp
echo "== p1" && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE --kernel-trace -d /tmp/a1 -o run --output-format csv -- python3 "$R/scripts/aes_enc_time.py" > "$R/$O/p1.log" 2>&1 || rc=$?
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 "$R/$O/p1.log"; exit $rc; }
echo "== p2" && timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d /tmp/a2 -o run --output-format csv -- python3 "$R/scripts/aes_enc_time.py" > "$R/$O/p2.log" 2>&1 || rc=$?
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 "$R/$O/p2.log"; exit $rc; }
cd "$R"
find /tmp/a1 -name "*counter_collection.csv" -exec cp {} $O/p1_counters.csv \;
find /tmp/a2 -name "*counter_collection.csv" -exec cp {} $O/p2_counters.csv \;
echo "== rc $rc"
exit $rc
