#!/bin/bash
# Round-5 pass af: member-sum width (DN_SUM_WIDE 2, product) vs 1 and 4:
# the sum's GPU tests, then an alternating A/B of the kernel.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05af}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest" && timeout -k 10 300 python -u -m pytest tests/test_gpu_agg.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -1 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head -5; exit $rc; }
for r in 1 2 3; do
  for v in product sum1 sum4; do
    if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
    timeout -k 10 120 python scripts/sum_time.py >> $O/sum.jsonl 2>> $O/sum.err || { rc=$?; break 2; }
    tail -1 $O/sum.jsonl
  done
done
echo "== rc $rc"
exit $rc
