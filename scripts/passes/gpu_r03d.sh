#!/bin/bash
# Round-3 A/B pass 4: device-PRNG split with paired ChaCha blocks (vs lib/ab/libdn_shamir_prngx1.so)
# and the AES envelope with base64-only hex digits (vs the v_perm variant), after their GPU tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03d}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_aes.py tests/test_gpu_prng.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -1 $O/pytest.log
for i in 1 2; do
  [ $rc = 0 ] || break
  echo "== prng x1 $i" && DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_prngx1.so" timeout -k 10 120 python scripts/prng_ab.py >> $O/prng_ab.jsonl 2>> $O/ab.err || { rc=$?; break; }
  echo "== prng x2 $i" && timeout -k 10 120 python scripts/prng_ab.py >> $O/prng_ab.jsonl 2>> $O/ab.err || { rc=$?; break; }
  echo "== aes perm $i" && DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_perm.so" timeout -k 10 120 python scripts/aes_ab.py >> $O/aes_ab.jsonl 2>> $O/ab.err || { rc=$?; break; }
  echo "== aes new $i" && timeout -k 10 120 python scripts/aes_ab.py >> $O/aes_ab.jsonl 2>> $O/ab.err || { rc=$?; break; }
done
cat $O/prng_ab.jsonl $O/aes_ab.jsonl
echo "== rc $rc"
exit $rc
