#!/bin/bash
# MT19937 device draw: parity tests, rate, kernel profile (each step time-limited, first failure ends it).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== mt tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q -k "mt or draw or config4 or sharded or fused or digest or reference" --timeout 300 --timeout-method thread > gpurun_out/pytest_mt.log 2>&1 \
&& echo "== rate" && timeout -k 10 200 python scripts/mt_draw_rate.py > gpurun_out/mt_draw_rate.json 2> gpurun_out/mt_draw_rate.err \
&& echo "== rocprof" && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_mt -o run --output-format csv -- python3 "${GRAFT_REPO_ROOT:-/root/repo}/scripts/mt_draw_rate.py" > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/rocprof_mt.log" 2>&1 \
&& cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/prof_mt && find /tmp/prof_mt -name "*.csv" -exec cp {} gpurun_out/prof_mt/ \; \
&& echo "== done"
rc=$?
tail -5 gpurun_out/pytest_mt.log 2>/dev/null
cat gpurun_out/mt_draw_rate.json 2>/dev/null
exit $rc
