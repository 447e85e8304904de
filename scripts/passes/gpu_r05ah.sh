#!/bin/bash
# Round-5 pass ah: member-sum width (DN_SUM_WIDE 4, product) vs 2 and 8, with
# the sum's GPU tests; then the headline reconstruct under the tuning
# library's wave schedules (DN_TILE_MAP 0 cyclic, 1 XCD, 3 coop), alternating.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05ah}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest" && timeout -k 10 300 python -u -m pytest tests/test_gpu_agg.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -1 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head -5; exit $rc; }
for r in 1 2 3; do
  for v in product sum2 sum8; do
    if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
    timeout -k 10 120 python scripts/sum_time.py >> $O/sum.jsonl 2>> $O/sum.err || { rc=$?; break 2; }
    tail -1 $O/sum.jsonl
  done
done
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
export DN_SHAMIR_LIB="$R/delta-node_amd/lib/libdn_shamir_tuning.so"
for r in 1 2 3; do
  for m in 0 1 3; do
    DN_TILE_MAP=$m timeout -k 10 120 python scripts/recon_time.py >> $O/recon.jsonl 2>> $O/recon.err || { rc=$?; break 2; }
    tail -1 $O/recon.jsonl
  done
done
echo "== rc $rc"
exit $rc
