#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r06v
mkdir -p $O
rc=0
echo "== pytest aes (variant)" && DN_SHAMIR_LIB=delta-node_amd/lib/ab/libdn_shamir_coal2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_aes.py -x -q --timeout 240 --timeout-method thread > $O/pytest_aes.log 2>&1 || rc=$?
tail -2 $O/pytest_aes.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error|assert" $O/pytest_aes.log | head -5; exit $rc; }
for round in 1 2 3 4; do
  for lib in libdn_shamir.so ab/libdn_shamir_coal2.so; do
    DN_SHAMIR_LIB=delta-node_amd/lib/$lib timeout -k 10 120 python scripts/aes_enc_time.py >> $O/aes_ab.jsonl 2>> $O/aes_ab.err || { rc=$?; echo "== $lib rc $rc"; tail -3 $O/aes_ab.err; exit $rc; }
  done
done
cat $O/aes_ab.jsonl
echo "== rc $rc"
exit $rc
