#!/bin/bash
# Round-4 pass b: the share-block allocator tests, the default bench line
# (share blocks from memory.share_block), and the rocprof kernel summary of the
# same bench command.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04b}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== test" && timeout -k 10 300 python -u -m pytest tests/test_gpu_memory.py tests/test_gpu_bench.py -x -v -m gpu --timeout 280 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
echo "== bench" && timeout -k 10 500 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || rc=$?
cut -c1-600 $O/bench_n1.json
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/bench_n1.err; exit $rc; }
echo "== rocprof" && cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_b -o run --output-format csv -- python3 "$R/bench.py" --cpu-budget 0 > "$R/$O/bench_under_rocprof.json" 2> "$R/$O/rocprof.err" || rc=$?
cd "$R" && mkdir -p $O/prof && find /tmp/prof_b -name "*stats.csv" -exec cp {} $O/prof/ \;
echo "== rc $rc"
exit $rc
