#!/bin/bash
# Round-3 A/B pass: AES envelope (SDWA-addressed rounds vs v_perm, lib/ab/libdn_shamir_perm.so)
# after its GPU tests, then the fused draw + split's store cache policy (tuning library).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03b}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== aes tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_aes.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_aes.log 2>&1 || rc=$?
tail -2 $O/pytest_aes.log
for i in 1 2; do
  [ $rc = 0 ] || break
  echo "== aes perm $i" && DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_perm.so" timeout -k 10 120 python scripts/aes_ab.py >> $O/aes_ab.jsonl 2>> $O/aes_ab.err || { rc=$?; break; }
  echo "== aes sdwa $i" && timeout -k 10 120 python scripts/aes_ab.py >> $O/aes_ab.jsonl 2>> $O/aes_ab.err || { rc=$?; break; }
done
if [ $rc = 0 ]; then
  echo "== mt aux" && timeout -k 10 200 python scripts/mt_aux_probe.py > $O/mt_aux.json 2> $O/mt_aux.err || rc=$?
fi
cat $O/aes_ab.jsonl; cut -c1-400 $O/mt_aux.json
echo "== rc $rc"
exit $rc
