#!/bin/bash
# MT jump-table layout A/B (tuning build): wall times, then rocprof kernel stats of the same script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out/mtab
export TMPDIR=/tmp
echo "== ab" && timeout -k 10 200 python scripts/mt_jump_ab.py > gpurun_out/mtab/ab.jsonl 2> gpurun_out/mtab/ab.err \
&& echo "== rocprof" && cd /tmp && REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_ab -o run --output-format csv -- python3 "$R/scripts/mt_jump_ab.py" > "$R/gpurun_out/mtab/rocprof.log" 2>&1 \
&& cd "$R" && find /tmp/prof_ab -name "*kernel_trace.csv" -exec cp {} gpurun_out/mtab/ \; \
&& echo "== done"
rc=$?
cat gpurun_out/mtab/ab.jsonl 2>/dev/null
exit $rc
