#!/bin/bash
# Round-5 pass m: AES decrypt with three interleaved blocks and the templated
# member sum — their GPU tests, then A/Bs in alternating processes against
# lib/ab/libdn_shamir_aesdec1.so and lib/ab/libdn_shamir_presum.so.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05m}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest aes+agg" && timeout -k 10 300 python -u -m pytest tests/test_gpu_aes.py tests/test_gpu_agg.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head -5; exit $rc; }
for r in 1 2; do
  for v in product aesdec1; do
    if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
    echo "== aes $v $r" && timeout -k 10 120 python scripts/aes_enc_time.py >> $O/aes.jsonl 2>> $O/aes.err || { rc=$?; break 2; }
    tail -1 $O/aes.jsonl
  done
  for v in product presum; do
    if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
    echo "== sum $v $r" && timeout -k 10 120 python scripts/sum_time.py >> $O/sum.jsonl 2>> $O/sum.err || { rc=$?; break 2; }
    tail -1 $O/sum.jsonl
  done
done
unset DN_SHAMIR_LIB
echo "== rc $rc"
exit $rc
