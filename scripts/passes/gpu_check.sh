#!/bin/bash
# GPU-box check: smoke, gpu parity tests, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; steps are chained so that the first
# failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
&& echo "== pytest gpu" && timeout -k 10 ${PYTEST_TIMEOUT:-600} python -m pytest tests -x -q -m "gpu${PYTEST_EXTRA:+ and $PYTEST_EXTRA}" > gpurun_out/pytest_gpu.log 2>&1 \
&& echo "== bench" && timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err \
&& echo "== rocprof" && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run --output-format csv -- python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --cpu-budget 0 --steps 20 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/rocprof.log" 2>&1 \
&& cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/prof_$TAG && find /tmp/prof_$TAG -name "*.csv" -exec cp {} gpurun_out/prof_$TAG/ \; \
&& echo "== done"
rc=$?
tail -3 gpurun_out/pytest_gpu.log 2>/dev/null
cat gpurun_out/bench.json 2>/dev/null
exit $rc
