#!/bin/bash
# Round-6 full pass: smoke, the whole GPU suite, make_shares_vec per-call
# times (caller buffer and the default pooled output), the default bench line
# (cold first call included), the rocprof kernel summary of the same bench
# command, then the HBM traffic passes (separate --pmc runs, kernel trace only).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06full}
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
echo "== msv overhead" && timeout -k 10 200 python scripts/msv_overhead.py > $O/msv_overhead.json 2>&1 || rc=$?
cut -c1-600 $O/msv_overhead.json
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
echo "== bench" && timeout -k 10 700 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || rc=$?
cut -c1-300 $O/bench_n1.json
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/bench_n1.err; exit $rc; }
echo "== rocprof" && cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_full -o run --output-format csv -- python3 "$R/bench.py" --cpu-budget 0 --cold 0 > "$R/$O/bench_under_rocprof.json" 2> "$R/$O/rocprof.err" || rc=$?
cd "$R" && mkdir -p $O/prof && find /tmp/prof_full -name "*stats.csv" -exec cp {} $O/prof/ \;
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/rocprof.err; exit $rc; }
grep -E "split_kernel|reconstruct_kernel|mt_gen_pc|mt_jump" $O/prof/*kernel_stats.csv | cut -c1-200 | head -8
TAG=${T}_pmc SRC="round 6 (full pass)" bash scripts/passes/gpu_pmc_r04.sh || rc=$?
echo "== rc $rc"
exit $rc
