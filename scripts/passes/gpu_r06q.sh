#!/bin/bash
# Round-6 pass q: the 4-bit contiguous-table jump kernel (DN_MT_JUMP4B):
# parity, lone-call times per configuration, one kernel trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06q}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest" && timeout -k 10 300 python -u -m pytest tests/test_gpu_spec.py -x -q -k "four_bit or two_bit" --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error|assert" $O/pytest.log | head -8; exit $rc; }
timeout -k 10 200 python -u scripts/jump4b_probe.py > $O/probe.jsonl 2> $O/probe.err || rc=$?
cat $O/probe.jsonl
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/probe.err; exit $rc; }
cd /tmp && ROUNDS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/kt_q -o run --output-format csv -- python3 "$R/scripts/jump4b_probe.py" > "$R/$O/kt.jsonl" 2>&1 || rc=$?
cd "$R" && find /tmp/kt_q -name "*kernel_trace.csv" -exec cp {} $O/kt.csv \; && find /tmp/kt_q -name "*kernel_stats.csv" -exec cp {} $O/stats.csv \;
echo "== rc $rc"
exit $rc
