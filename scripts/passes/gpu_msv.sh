#!/bin/bash
# make_shares_vec per-call cost at several sizes (+ kernel trace), then the MT parity tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/msv
mkdir -p $O
export TMPDIR=/tmp
echo "== wall" && timeout -k 10 200 python scripts/msv_overhead.py > $O/wall.json 2> $O/wall.err \
&& echo "== trace" && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_msv -o run --output-format csv -- python3 "$R/scripts/msv_overhead.py" > "$R/$O/rocprof.log" 2>&1 \
&& cd "$R" && find /tmp/prof_msv -name "*kernel_trace.csv" -exec cp {} $O/ \; \
&& echo "== tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q -m gpu -k "mt or draw or fused or sharded or config4" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
&& echo "== done"
rc=$?
cat $O/wall*.json; tail -2 $O/pytest.log
exit $rc
