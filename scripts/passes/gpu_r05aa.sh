#!/bin/bash
# Round-5 pass aa: share-block pool events without the system-scope fence
# (product) vs with it (variant evfence): memory (stream-order) GPU tests,
# make_shares_vec back to back with the default pooled output (wall time per
# call, alternating processes), and the GPU gaps between calls of each.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05aa}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest" && timeout -k 10 400 python -u -m pytest tests/test_gpu_memory.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -1 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head -5; exit $rc; }
for r in 1 2 3; do
  for L in 24 20; do
    for v in product evfence; do
      if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
      timeout -k 10 120 python scripts/msv_loop_gaps.py $L >> $O/walls.jsonl 2>> $O/walls.err || { rc=$?; break 3; }
      tail -1 $O/walls.jsonl
    done
  done
done
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
for v in product evfence; do
  if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
  cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/g_$v -o run --output-format csv -- python3 "$R/scripts/msv_loop_gaps.py" 24 > "$R/$O/trace_wall_$v.json" 2> "$R/$O/trace_$v.err" || rc=$?
  cd "$R"
  [ $rc -ne 0 ] && { echo "== rc $rc"; tail -3 $O/trace_$v.err; exit $rc; }
  python3 scripts/msv_loop_gaps.py --summary /tmp/g_$v > $O/gaps_$v.json && cut -c1-300 $O/gaps_$v.json
done
echo "== rc $rc"
exit $rc
