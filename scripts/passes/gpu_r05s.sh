#!/bin/bash
# Round-5 pass s: decode reads of the half-line transposed text
# (DN_AES_DEC_COAL=2, variant deccoal2) against the product (encrypt with
# the two-stage transpose by default): AES GPU tests on both, then the
# encrypt/decrypt kernel A/B, alternating processes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05s}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest aes" && timeout -k 10 300 python -u -m pytest tests/test_gpu_aes.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head -5; exit $rc; }
echo "== pytest aes coal2" && DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_deccoal2.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_aes.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_coal2.log 2>&1 || rc=$?
tail -2 $O/pytest_coal2.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest_coal2.log | head -5; exit $rc; }
for r in 1 2 3; do
  for v in product ${VARIANTS:-deccoal2}; do
    if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
    echo "== $v $r" && timeout -k 10 120 python scripts/aes_enc_time.py >> $O/aes.jsonl 2>> $O/aes.err || { rc=$?; break 2; }
    tail -1 $O/aes.jsonl | cut -c1-200
  done
done
echo "== rc $rc"
exit $rc
