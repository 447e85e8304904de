#!/bin/bash
# Round-3 pass n: MT parity tests of the product library, then the generation
# rate by direction (tuning library, DN_MT_BACK = 0 all forward, 1 product:
# even substreams backward, 2 every inner substream backward): kernel stats
# of scripts/mt_draw_rate.py under each.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03n}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "mt or draw or fused or digest" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
for mode in 0 1 2; do
  [ $rc = 0 ] || break
  echo "== mode $mode"
  export DN_SHAMIR_LIB=$R/delta-node_amd/lib/libdn_shamir_tuning.so DN_MT_BACK=$mode
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_back_$mode -o run --output-format csv -- python3 "$R/scripts/mt_draw_rate.py" > "$R/$O/mt_draw_rate_$mode.json" 2> "$R/$O/rocprof_$mode.err") || rc=$?
  find /tmp/prof_back_$mode -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$mode.csv \;
  grep -h "mt_gen\|mt_jump" $O/kernel_stats_$mode.csv | cut -d, -f1-4
done
echo "== rc $rc"
exit $rc
