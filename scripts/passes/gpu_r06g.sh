#!/bin/bash
# Round-6 pass g: the speculative next-call jump levels (DN_MT_SPEC): parity
# (tests/test_gpu_spec.py and the MT/fused parity tests), then an
# alternating-process A/B of make_shares_vec (scripts/msv_ab.py) product vs a
# no-speculation build, and one kernel trace of each for the timeline.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06g}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest spec" && timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_parity.py -x -q -k "spec or mt_draw or fused or concurrent or retry or shard or two_wave" --timeout 240 --timeout-method thread > $O/pytest_spec.log 2>&1 || rc=$?
tail -2 $O/pytest_spec.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error|assert" $O/pytest_spec.log | head -8; exit $rc; }
for round in 1 2 3; do
  for lib in libdn_shamir.so ab/libdn_shamir_nospec.so; do
    DN_SHAMIR_LIB=delta-node_amd/lib/$lib timeout -k 10 180 python scripts/msv_ab.py >> $O/msv_ab.jsonl 2>> $O/msv_ab.err || { rc=$?; echo "== $lib rc $rc"; tail -3 $O/msv_ab.err; exit $rc; }
  done
done
cut -c1-400 $O/msv_ab.jsonl
for lib in libdn_shamir.so ab/libdn_shamir_nospec.so; do
  tag=$(basename $lib .so)
  cd /tmp && DN_SHAMIR_LIB=$R/delta-node_amd/lib/$lib timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/kt_$tag -o run --output-format csv -- python3 "$R/scripts/msv_ab.py" > "$R/$O/kt_$tag.json" 2>&1 || rc=$?
  cd "$R" && find /tmp/kt_$tag -name "*kernel_trace.csv" -exec cp {} $O/kt_$tag.csv \;
  [ $rc -ne 0 ] && { echo "== rc $rc"; tail -3 $O/kt_$tag.json; exit $rc; }
done
echo "== rc $rc"
exit $rc
