#!/bin/bash
# Round-3 pass q: a small bench (2^20, rows on) as a quick check of every
# row's code, the default bench line, the rocprof kernel stats of the
# headline bench, and one make_shares_vec call's GPU timeline (kernel +
# memory-copy trace).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03q}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== small bench" && timeout -k 10 300 python bench.py --log2n 20 --steps 3 --warmup 1 --config4 0 --config5 0 --cpu-budget 0 > $O/bench_small.json 2> $O/bench_small.err || rc=$?
[ $rc = 0 ] && cut -c1-300 $O/bench_small.json
if [ $rc = 0 ]; then
  echo "== bench" && timeout -k 10 500 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || rc=$?
  cut -c1-600 $O/bench_n1.json
fi
if [ $rc = 0 ]; then
  echo "== rocprof" && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_bench -o run \
      --output-format csv -- python3 "$R/bench.py" --cpu-budget 0 --rows 0 --config4 0 --config5 0 \
      > "$R/$O/bench_under_rocprof.json" 2> "$R/$O/rocprof.err") || rc=$?
  find /tmp/prof_bench -name "*kernel_stats.csv" -exec cp {} $O/rocprof_kernel_stats.csv \;
  head -8 $O/rocprof_kernel_stats.csv | cut -c1-160
fi
if [ $rc = 0 ]; then
  echo "== msv trace" && (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/prof_msv -o run \
      --output-format csv -- python3 "$R/scripts/msv_trace.py" > "$R/$O/msv_wall.json" 2> "$R/$O/msv_trace.err") || rc=$?
  python3 scripts/msv_trace_summary.py /tmp/prof_msv > $O/msv_timeline.json 2>> $O/msv_trace.err || true
  cat $O/msv_wall.json; head -c 3000 $O/msv_timeline.json
fi
echo "== rc $rc"
exit $rc
