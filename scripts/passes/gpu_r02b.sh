#!/bin/bash
# Round-2 full GPU pass: all gpu tests, smoke(), the default bench line, and
# the rocprofv3 kernel summary of the same bench command.  Each GPU step has
# its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gpu" && timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
&& echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
&& echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
&& echo "== rocprof bench" && R=$PWD && cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_bench -o run --output-format csv -- python3 "$R/bench.py" --cpu-budget 0 > "$R/gpurun_out/bench_prof.json" 2> "$R/gpurun_out/bench_prof.err" && mkdir -p "$R/gpurun_out/prof_bench" && cp -r /tmp/prof_bench/. "$R/gpurun_out/prof_bench/" && cd "$R" \
&& echo "== done"
rc=$?
tail -3 gpurun_out/pytest_gpu.log 2>/dev/null
exit $rc
