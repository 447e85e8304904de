#!/bin/bash
# Round-5 pass y: the MT jump kernel's polynomial words by scalar loads, one
# wait per run of 11 Horner steps (DN_MT_JUMP_SMEM, product) against a vector
# load per step (variant smem0): MT / parity / sharded GPU tests, then
# make_shares_vec wall time per call (alternating processes) and the kernel
# summaries of both builds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05y}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest" && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_memory.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -1 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head -5; exit $rc; }
for r in 1 2 3; do
  for L in 24 20; do
    for v in product smem0; do
      if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
      timeout -k 10 120 python scripts/msv_loop_gaps.py $L >> $O/walls.jsonl 2>> $O/walls.err || { rc=$?; break 3; }
      tail -1 $O/walls.jsonl
    done
  done
done
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
for v in product smem0; do
  if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
  cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d /tmp/jp_$v -o run --output-format csv -- python3 "$R/scripts/msv_loop_gaps.py" 24 > "$R/$O/prof_wall_$v.json" 2> "$R/$O/prof_$v.err" || rc=$?
  cd "$R"
  [ $rc -ne 0 ] && { echo "== rc $rc"; tail -3 $O/prof_$v.err; exit $rc; }
  find /tmp/jp_$v -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$v.csv \;
  grep -E "mt_jump|mt_gen_pc|mt_combine" $O/kernel_stats_$v.csv | cut -c1-160
done
echo "== rc $rc"
exit $rc
