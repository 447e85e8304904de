#!/bin/bash
# Round-3 A/B pass 3: MT draw (ring generator + prefetched secrets) vs the
# round-2 library, AES envelope (SDWA + prefetched loads) vs the v_perm variant.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03c}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== aes tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_aes.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_aes.log 2>&1 || rc=$?
tail -1 $O/pytest_aes.log
if [ $rc = 0 ]; then TAG=${TAG:-r03c}_mt bash scripts/ab_msv.sh > $O/ab_msv.out 2>&1 || rc=$?; tail -22 $O/ab_msv.out; fi
for i in 1 2; do
  [ $rc = 0 ] || break
  echo "== aes perm $i" && DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_perm.so" timeout -k 10 120 python scripts/aes_ab.py >> $O/aes_ab.jsonl 2>> $O/aes_ab.err || { rc=$?; break; }
  echo "== aes new $i" && timeout -k 10 120 python scripts/aes_ab.py >> $O/aes_ab.jsonl 2>> $O/aes_ab.err || { rc=$?; break; }
done
cat $O/aes_ab.jsonl
echo "== rc $rc"
exit $rc
