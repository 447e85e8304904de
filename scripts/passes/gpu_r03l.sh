#!/bin/bash
# Round-3 pass l: the PRNG split (two / four tiles' top-limb blocks per pass,
# its own launch-bounded kernel at 80 VGPRs) against one tile per pass
# (lib/ab/libdn_shamir_notp.so), three alternations, after the PRNG tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03l}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== prng tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_prng.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_prng.log 2>&1 || rc=$?
tail -2 $O/pytest_prng.log
for rep in 1 2 3; do
  for v in ab/libdn_shamir_notp.so libdn_shamir.so; do
    [ $rc = 0 ] || break
    echo "== prng $v $rep"
    DN_SHAMIR_LIB=$R/delta-node_amd/lib/$v timeout -k 10 120 python scripts/prng_ab.py >> $O/prng_tp.jsonl 2>> $O/prng.err || rc=$?
  done
done
cat $O/prng_tp.jsonl
echo "== rc $rc"
exit $rc
