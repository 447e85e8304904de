#!/bin/bash
# Round-6 pass n: the two-bit jump kernel (mt_jump2_kernel<4>, 11 KB table):
# parity in place of the direct level (DN_MT_SPEC_PROBE=5), then loop times
# with no levels (1), the product sequence (0), the levels by the two-bit
# kernel alone (5) and beside the generation on a side stream (4); one trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06n}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest" && timeout -k 10 300 python -u -m pytest tests/test_gpu_spec.py -x -q -k "two_bit" --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error|assert" $O/pytest.log | head -8; exit $rc; }
MODES=0,1,5,4 ROUNDS=2 timeout -k 10 240 python -u scripts/spec_probe.py > $O/spec_probe.jsonl 2> $O/spec_probe.err || rc=$?
cat $O/spec_probe.jsonl
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/spec_probe.err; exit $rc; }
cd /tmp && MODES=4,5 ROUNDS=1 timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/kt_n -o run --output-format csv -- python3 "$R/scripts/spec_probe.py" > "$R/$O/kt.jsonl" 2>&1 || rc=$?
cd "$R" && find /tmp/kt_n -name "*kernel_trace.csv" -exec cp {} $O/kt.csv \;
echo "== rc $rc"
exit $rc
