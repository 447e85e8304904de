#!/bin/bash
# Round-5 pass an: reconstruct with one quarter loaded ahead (product) vs two (DN_RECON_PF=2, variant pf2)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05an}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for v in product pf2; do
  if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
  echo "== pytest $v" && timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_agg.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || rc=$?
  tail -1 $O/pytest_$v.log
  [ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest_$v.log | head -5; exit $rc; }
done
for r in 1 2 3; do
  for v in product pf2; do
    if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
    timeout -k 10 120 python scripts/recon_time.py >> $O/recon.jsonl 2>> $O/recon.err || { rc=$?; break 2; }
    tail -1 $O/recon.jsonl
  done
done
echo "== rc $rc"
exit $rc
