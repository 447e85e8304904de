#!/bin/bash
# Round-6 pass t: the beside kernel with 3-bit chunks (DN_MT_BESIDE_CB=3, the
# product candidate) vs 2-bit (lib/ab/libdn_shamir_cb2.so): parity, then 2^24
# loops and lone calls (scripts/msv_loop.py), alternating processes; one
# kernel trace of the product's loop.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06t}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest spec" && timeout -k 10 500 python -u -m pytest tests/test_gpu_spec.py -x -q --timeout 240 --timeout-method thread > $O/pytest_spec.log 2>&1 || rc=$?
tail -2 $O/pytest_spec.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error|assert" $O/pytest_spec.log | head -8; exit $rc; }
for round in 1 2 3 4; do
  for lib in libdn_shamir.so ab/libdn_shamir_cb2.so; do
    SIZES=24 DN_SHAMIR_LIB=delta-node_amd/lib/$lib timeout -k 10 120 python scripts/msv_loop.py >> $O/msv_loop.jsonl 2>> $O/msv_loop.err || { rc=$?; echo "== $lib rc $rc"; tail -3 $O/msv_loop.err; exit $rc; }
  done
done
cut -c1-330 $O/msv_loop.jsonl
cd /tmp && SIZES=24 timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/kt_t -o run --output-format csv -- python3 "$R/scripts/msv_loop.py" > "$R/$O/kt_loop.json" 2>&1 || rc=$?
cd "$R" && find /tmp/kt_t -name "*kernel_trace.csv" -exec cp {} $O/kt_loop.csv \;
echo "== rc $rc"
exit $rc
