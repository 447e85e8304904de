#!/bin/bash
# Round-6 pass c: the fused draw + split's generation time against the
# substreams in flight (scripts/mt_gen_scaling.py, tuning build), wall times
# and the rocprof kernel summary of the same run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06c}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rc=0
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_scal -o run --output-format csv -- python3 "$R/scripts/mt_gen_scaling.py" > "$R/$O/scaling.jsonl" 2> "$R/$O/scaling.err" || rc=$?
cd "$R" && mkdir -p $O/prof && find /tmp/prof_scal -name "*.csv" -exec cp {} $O/prof/ \;
cat $O/scaling.jsonl | cut -c1-200
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/scaling.err; exit $rc; }
echo "== rc $rc"
exit $rc
