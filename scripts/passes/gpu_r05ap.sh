#!/bin/bash
# Round-5 pass ap: the default bench line twice (fresh processes) on one more
# box, HEAD, for the spread across boxes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05ap}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for r in 1 2; do
  echo "== bench $r" && timeout -k 10 700 python bench.py > $O/bench_$r.json 2> $O/bench_$r.err || { rc=$?; tail -3 $O/bench_$r.err; break; }
  cut -c1-200 $O/bench_$r.json
done
echo "== rc $rc"
exit $rc
