#!/bin/bash
# Round-3 pass 7: AES encrypt with the three keystream blocks of a unit run
# interleaved (DN_AES_NB 3 = product, 2, 1 = previous) A/B'd twice in
# alternation, the AES and MT GPU tests on the product library.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03g}
mkdir -p $O
export TMPDIR=/tmp
rc=0
L=delta-node_amd/lib
for rep in 1 2; do
  for v in ${LIBS:-ab/libdn_shamir_nb1.so ab/libdn_shamir_nb2.so libdn_shamir.so}; do
    [ $rc = 0 ] || break
    echo "== aes $v $rep"
    DN_SHAMIR_LIB=$R/$L/$v timeout -k 10 120 python scripts/aes_ab.py >> $O/aes_ab.jsonl 2>> $O/aes_ab.err || rc=$?
  done
done
cat $O/aes_ab.jsonl
if [ $rc = 0 ]; then
  echo "== tests"
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_aes.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || rc=$?
  tail -3 $O/pytest.log
fi
echo "== rc $rc"
exit $rc
