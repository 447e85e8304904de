#!/bin/bash
# MiMC7 kernels: GPU tests, then the bench rows (incl. data commitment at 2^15 / 2^20 rows) and kernel trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/mimc
mkdir -p $O
export TMPDIR=/tmp
echo "== tests" && timeout -k 10 400 python -u -m pytest tests/test_mimc7.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
&& echo "== rows" && ROWS=rows timeout -k 10 300 python scripts/rows_probe.py > $O/rows.json 2> $O/rows.err \
&& echo "== trace" && cd /tmp && ROWS=rows timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_mimc -o run --output-format csv -- python3 "$R/scripts/rows_probe.py" > "$R/$O/rocprof.log" 2>&1 \
&& cd "$R" && find /tmp/prof_mimc -name "*kernel_trace.csv" -exec cp {} $O/ \; \
&& echo "== done"
rc=$?
tail -3 $O/pytest.log
exit $rc
