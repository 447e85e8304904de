#!/bin/bash
# Round-5 pass r: hex table base folded into the lane bits (DN_AES_HEX_BASE,
# product) and the two-stage half-line text transpose (DN_AES_HEX_COAL=2,
# variant aescoal2): AES GPU tests on both, then encrypt/decrypt kernel A/B
# against the previous build (aeshb0), alternating processes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05r}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest aes" && timeout -k 10 300 python -u -m pytest tests/test_gpu_aes.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head -5; exit $rc; }
echo "== pytest aes coal2" && DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_aescoal2.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_aes.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_coal2.log 2>&1 || rc=$?
tail -2 $O/pytest_coal2.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest_coal2.log | head -5; exit $rc; }
for r in 1 2 3; do
  for v in product ${VARIANTS:-aeshb0 aescoal2}; do
    if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
    echo "== $v $r" && timeout -k 10 120 python scripts/aes_enc_time.py >> $O/aes.jsonl 2>> $O/aes.err || { rc=$?; break 2; }
    tail -1 $O/aes.jsonl | cut -c1-200
  done
done
echo "== rc $rc"
exit $rc
