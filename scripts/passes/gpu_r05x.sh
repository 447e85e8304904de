#!/bin/bash
# Round-5 pass x: one-pass decrypt with the coalesced transposed text reads
# (decrypt_fused_kernel, DN_AES_DEC_SPLIT=2; DEC_NB 1 and 3): AES GPU tests on
# both variants, then the encrypt/decrypt kernel A/B against the product's
# two passes, alternating processes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05x}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for v in decf1 decf3; do
  echo "== pytest aes $v" && DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_aes.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || rc=$?
  tail -1 $O/pytest_$v.log
  [ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest_$v.log | head -5; exit $rc; }
done
for r in 1 2 3; do
  for v in product decf1 decf3; do
    if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
    echo "== $v $r" && timeout -k 10 120 python scripts/aes_enc_time.py >> $O/aes.jsonl 2>> $O/aes.err || { rc=$?; break 2; }
    tail -1 $O/aes.jsonl | cut -c1-200
  done
done
echo "== rc $rc"
exit $rc
