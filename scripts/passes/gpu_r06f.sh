#!/bin/bash
# Round-6 pass f: the speculative next-call jump level's potential
# (scripts/spec_probe.py, DN_MT_SPEC_PROBE in the tuning build): loop times per
# mode, then one kernel trace of modes 0 and 2 for the timeline.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06f}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== spec probe" && timeout -k 10 240 python -u scripts/spec_probe.py > $O/spec_probe.jsonl 2> $O/spec_probe.err || rc=$?
cat $O/spec_probe.jsonl
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/spec_probe.err; exit $rc; }
cd /tmp && MODES=0,2 ROUNDS=1 timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/kt_spec -o run --output-format csv -- python3 "$R/scripts/spec_probe.py" > "$R/$O/kt_spec.jsonl" 2>&1 || rc=$?
cd "$R" && find /tmp/kt_spec -name "*kernel_trace.csv" -exec cp {} $O/kt_spec.csv \;
echo "== rc $rc"
exit $rc
