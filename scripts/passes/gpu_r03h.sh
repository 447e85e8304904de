#!/bin/bash
# Round-3 pass h: backward generation of the even MT substreams A/B'd against
# the HEAD library (scripts/ab_msv.sh: MT parity tests, make_shares_vec wall
# time, kernel stats), then the VALU issue rates by encoding (tools/valu_rates).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03h}
mkdir -p $O
rc=0
TAG=${TAG:-r03h} BASE=${BASE:-HEAD} bash scripts/ab_msv.sh || rc=$?
if [ $rc = 0 ]; then
  echo "== valu rates" && timeout -k 10 120 tools/valu_rates > $O/valu_rates.jsonl 2>&1 || rc=$?
  cat $O/valu_rates.jsonl
fi
echo "== rc $rc"
exit $rc
