#!/bin/bash
# Round-6 pass h: speculation (DN_MT_SPEC) with the continuation policy:
# parity, then back-to-back loops and lone calls per size (scripts/msv_loop.py),
# product vs the no-speculation build, alternating processes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06h}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest spec" && timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_parity.py -x -q -k "spec or mt_draw or fused or concurrent or retry or shard or two_wave" --timeout 240 --timeout-method thread > $O/pytest_spec.log 2>&1 || rc=$?
tail -2 $O/pytest_spec.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error|assert" $O/pytest_spec.log | head -8; exit $rc; }
for round in 1 2 3; do
  for lib in libdn_shamir.so ab/libdn_shamir_nospec.so; do
    DN_SHAMIR_LIB=delta-node_amd/lib/$lib timeout -k 10 180 python scripts/msv_loop.py >> $O/msv_loop.jsonl 2>> $O/msv_loop.err || { rc=$?; echo "== $lib rc $rc"; tail -3 $O/msv_loop.err; exit $rc; }
  done
done
cut -c1-600 $O/msv_loop.jsonl
echo "== rc $rc"
exit $rc
