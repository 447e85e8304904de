#!/bin/bash
# Round-4 pass c: MT parity tests (direct jump level for <= 65 substreams,
# 2^8-draw substreams), the share-block allocator tests, make_shares_vec's
# GPU timeline at 2^12 / 2^16 / 2^24, then the default bench line and the
# rocprof kernel summary of the same bench command.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04c}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== test" && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_memory.py -x -v -m gpu -k "mt or fused or draw or memory or block or shares_vec or digest" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
echo "== msv trace"
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/msvtr -o run --output-format csv -- python3 "$R/scripts/msv_trace.py" 12 16 24 > "$R/$O/msv_trace.json" 2> "$R/$O/msv_trace.err" || rc=$?
cd "$R"
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
mkdir -p $O/msvtr && find /tmp/msvtr -name "*.csv" -exec cp {} $O/msvtr/ \;
python3 scripts/msv_trace_summary.py $O/msvtr 24 > $O/msv_timeline.json || true
cat $O/msv_trace.json
echo "== msv overhead" && timeout -k 10 200 python scripts/msv_overhead.py > $O/msv_overhead.json 2>&1 || rc=$?
cat $O/msv_overhead.json | cut -c1-800
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
echo "== bench" && timeout -k 10 500 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || rc=$?
cut -c1-600 $O/bench_n1.json
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/bench_n1.err; exit $rc; }
echo "== rocprof" && cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_c -o run --output-format csv -- python3 "$R/bench.py" --cpu-budget 0 > "$R/$O/bench_under_rocprof.json" 2> "$R/$O/rocprof.err" || rc=$?
cd "$R" && mkdir -p $O/prof && find /tmp/prof_c -name "*stats.csv" -exec cp {} $O/prof/ \;
echo "== rc $rc"
exit $rc
