#!/bin/bash
# Round-5 pass ae: the member sum with two 16-B pairs per lane and step
# (DN_SUM_WIDE, variant sumwide) against the product, alternating processes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05ae}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for r in 1 2 3; do
  for v in product sumwide; do
    if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
    timeout -k 10 120 python scripts/sum_time.py >> $O/sum.jsonl 2>> $O/sum.err || { rc=$?; break 2; }
    tail -1 $O/sum.jsonl
  done
done
echo "== rc $rc"
exit $rc
