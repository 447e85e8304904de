#!/bin/bash
# Round-4 pass h: (1) the share-block make_shares_vec mismatch of pass g
# (scripts/msv_block_debug.py, in-tree library and the library of 1729a03),
# (2) ChaCha first-column-round peel: PRNG parity tests, then prng_ab.py
# alternating in-tree vs lib/ab/libdn_shamir_HEAD.so, (3) the emission
# write-pattern probe (scripts/emit_pattern_probe.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04h}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== debug new" && TRIALS=8 timeout -k 10 180 python scripts/msv_block_debug.py > $O/debug_new.jsonl 2> $O/debug_new.err || rc=$?
cut -c1-700 $O/debug_new.jsonl
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/debug_new.err; exit $rc; }
echo "== debug 1729a03" && TRIALS=8 DN_SHAMIR_LIB=$R/delta-node_amd/lib/ab/libdn_shamir_1729a03.so timeout -k 10 180 python scripts/msv_block_debug.py > $O/debug_old.jsonl 2> $O/debug_old.err || rc=$?
cut -c1-700 $O/debug_old.jsonl
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/debug_old.err; exit $rc; }
echo "== prng tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_prng.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_prng.log 2>&1 || rc=$?
tail -2 $O/pytest_prng.log
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
for i in 1 2; do
  for v in new HEAD; do
    echo "== prng $v $i"
    if [ $v = new ]; then timeout -k 10 120 python scripts/prng_ab.py >> $O/prng_$v.jsonl 2>> $O/prng.err || rc=$?
    else DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_HEAD.so" timeout -k 10 120 python scripts/prng_ab.py >> $O/prng_$v.jsonl 2>> $O/prng.err || rc=$?; fi
    [ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/prng.err; exit $rc; }
  done
done
cat $O/prng_new.jsonl $O/prng_HEAD.jsonl
echo "== emit pattern" && timeout -k 10 300 python scripts/emit_pattern_probe.py > $O/emit_pattern.jsonl 2> $O/emit_pattern.err || rc=$?
cut -c1-600 $O/emit_pattern.jsonl
echo "== rc $rc"
exit $rc
