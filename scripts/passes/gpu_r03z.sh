#!/bin/bash
# Round-3 pass z: the bench-rows test, then the default bench line (rows with
# three output placements for make_shares_vec and the PRNG split).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03z}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== test" && timeout -k 10 200 python -u -m pytest tests/test_gpu_bench.py -x -q -m gpu -k rows_small --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
if [ $rc = 0 ]; then
  echo "== bench" && timeout -k 10 500 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || rc=$?
  cut -c1-300 $O/bench_n1.json
fi
echo "== rc $rc"
exit $rc
