#!/bin/bash
# Round-3 pass v: the one-copy MT scratch layout — MT / fused / sharded GPU
# tests and the small-bench rows test, one make_shares_vec call's GPU
# timeline, then the level-B part-count sweep (scripts/passes/gpu_r03u.sh).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03v}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== tests" && timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_bench.py -x -q -m gpu -k "mt or draw or fused or sharded or config4 or digest or bench" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
if [ $rc = 0 ]; then
  echo "== msv trace" && (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/prof_msv -o run \
      --output-format csv -- python3 "$R/scripts/msv_trace.py" > "$R/$O/msv_wall.json" 2> "$R/$O/msv_trace.err") || rc=$?
  python3 scripts/msv_trace_summary.py /tmp/prof_msv > $O/msv_timeline.json 2>> $O/msv_trace.err || true
  cat $O/msv_wall.json
fi
if [ $rc = 0 ]; then TAG=${TAG:-r03v}/parts bash scripts/passes/gpu_r03u.sh || rc=$?; fi
echo "== rc $rc"
exit $rc
