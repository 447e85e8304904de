#!/bin/bash
# Round-3 final pass: full `pytest -m gpu`, smoke, the default bench line,
# rocprof kernel stats of the headline bench, then a 4-rank gloo rehearsal of
# `bench.py --gpus 4` on the one GPU (config 4 at 2^22).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03y}
mkdir -p $O
export TMPDIR=/tmp
rc=0
TAG=${TAG:-r03y} STAGES=tests,smoke,bench,prof bash scripts/passes/gpu_r03.sh || rc=$?
if [ $rc = 0 ]; then
  echo "== 4-rank gloo rehearsal" && DN_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 4 --steps 5 --warmup 2 \
      --rows 0 --config5 0 --cpu-budget 0 --config4 1 --config4-log2n 22 > $O/bench4_gloo.json 2> $O/bench4_gloo.err || rc=$?
  cut -c1-800 $O/bench4_gloo.json
fi
echo "== rc $rc"
exit $rc
