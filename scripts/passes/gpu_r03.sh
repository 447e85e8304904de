#!/bin/bash
# Round-3 GPU pass: full `pytest -m gpu`, smoke, the default bench line, and
# (STAGES contains "prof") the rocprofv3 kernel stats of the headline bench.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03}
mkdir -p $O
export TMPDIR=/tmp
STAGES="${STAGES:-tests,smoke,bench}"
run() { case ",$STAGES," in *",$1,"*) return 0;; *) return 1;; esac; }
rc=0
if run tests; then
  echo "== tests" && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu ${PYTEST_K:+-k "$PYTEST_K"} \
      --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
  tail -3 $O/pytest_gpu.log
fi
if [ $rc = 0 ] && run smoke; then
  echo "== smoke" && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || rc=$?
  tail -2 $O/smoke.log
fi
if [ $rc = 0 ] && run bench; then
  echo "== bench" && timeout -k 10 500 python bench.py ${BENCH_ARGS} > $O/bench_n1.json 2> $O/bench_n1.err || rc=$?
  cut -c1-1500 $O/bench_n1.json
fi
if [ $rc = 0 ] && run prof; then
  echo "== rocprof" && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_bench -o run \
      --output-format csv -- python3 "$R/bench.py" --cpu-budget 0 --rows 0 --config4 0 --config5 0 \
      > "$R/$O/bench_under_rocprof.json" 2> "$R/$O/rocprof.err") || rc=$?
  find /tmp/prof_bench -name "*kernel_stats.csv" -exec cp {} $O/rocprof_kernel_stats.csv \;
  head -12 $O/rocprof_kernel_stats.csv 2>/dev/null | cut -c1-200
fi
echo "== rc $rc"
exit $rc
