#!/bin/bash
# Round-3 pass 5: device-PRNG split A/B (tile secrets parked in LDS, paired
# ChaCha blocks) against lib/ab/libdn_shamir_prngx1.so (round-2 loop, single
# blocks) and lib/ab/libdn_shamir_prngx1s.so (new loop, single blocks); then
# the full GPU suite, smoke, the default bench line and its rocprof stats.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03e}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== prng tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_prng.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_prng.log 2>&1 || rc=$?
tail -1 $O/pytest_prng.log
for i in 1 2; do
  [ $rc = 0 ] || break
  for v in prngx1 prngx1s; do
    echo "== prng $v $i" && DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so" timeout -k 10 120 python scripts/prng_ab.py >> $O/prng_ab.jsonl 2>> $O/ab.err || { rc=$?; break; }
  done
  [ $rc = 0 ] || break
  echo "== prng new $i" && timeout -k 10 120 python scripts/prng_ab.py >> $O/prng_ab.jsonl 2>> $O/ab.err || { rc=$?; break; }
done
cut -c1-330 $O/prng_ab.jsonl
if [ $rc = 0 ]; then TAG=${TAG:-r03e}_full STAGES=tests,smoke,bench,prof bash scripts/passes/gpu_r03.sh || rc=$?; fi
echo "== rc $rc"
exit $rc
