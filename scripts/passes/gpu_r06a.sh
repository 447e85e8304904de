#!/bin/bash
# Round-6 first pass: smoke, the whole GPU suite, the default bench line.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06a}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || rc=$?
tail -1 $O/smoke.log
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -5; exit $rc; }
echo "== bench" && timeout -k 10 700 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || rc=$?
cut -c1-300 $O/bench_n1.json
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/bench_n1.err; exit $rc; }
echo "== rc $rc"
exit $rc
