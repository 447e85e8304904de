#!/bin/bash
# Round-3 pass k: (1) the jump step with the table reads ahead of f^64's
# permutes (product) against DN_JUMP_PIPE=0 (scripts/ab_msv.sh, BASE=nopipe);
# (2) the PRNG split with two / four tiles' top-limb blocks per pass (product)
# against one (lib/ab/libdn_shamir_notp.so), alternating, after the PRNG tests;
# (3) the PRNG grid-cap sweep (scripts/passes/gpu_r03j.sh).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03k}
mkdir -p $O
export TMPDIR=/tmp
rc=0
TAG=${TAG:-r03k}/msv BASE=nopipe bash scripts/ab_msv.sh || rc=$?
if [ $rc = 0 ]; then
  echo "== prng tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_prng.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_prng.log 2>&1 || rc=$?
  tail -2 $O/pytest_prng.log
fi
for rep in 1 2 3; do
  for v in ab/libdn_shamir_notp.so libdn_shamir.so; do
    [ $rc = 0 ] || break
    echo "== prng $v $rep"
    DN_SHAMIR_LIB=$R/delta-node_amd/lib/$v timeout -k 10 120 python scripts/prng_ab.py >> $O/prng_tp.jsonl 2>> $O/prng.err || rc=$?
  done
done
cat $O/prng_tp.jsonl
if [ $rc = 0 ]; then TAG=${TAG:-r03k}/cap CAPS="0 512 1024 2048 4096" bash scripts/passes/gpu_r03j.sh || rc=$?; fi
echo "== rc $rc"
exit $rc
