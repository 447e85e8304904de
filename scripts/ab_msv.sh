#!/bin/bash
# A/B of the MT19937 device draw: the baseline library lib/ab/libdn_shamir_${BASE}.so
# (make ab REF=...) against the in-tree library.  First the MT / fused parity
# tests of the in-tree library, then make_shares_vec per-call wall time
# (alternating processes), then the kernel stats of scripts/mt_draw_rate.py
# (draw alone = mt_gen_kernel<0>, fused draw + split = mt_gen_kernel<3>, 2^24)
# under each library.  Each GPU step has its own time limit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-abmsv}
mkdir -p $O
export TMPDIR=/tmp
BASE_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_${BASE:-HEAD}.so"
rc=0
if [ -z "$NOTEST" ]; then
  echo "== tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q -m gpu -k "mt or draw or fused or sharded or config4 or digest" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
  tail -2 $O/pytest.log
fi
for i in 1 2; do
  [ $rc = 0 ] || break
  echo "== base $i" && DN_SHAMIR_LIB="$BASE_LIB" timeout -k 10 120 python scripts/msv_overhead.py >> $O/wall_base.jsonl 2>> $O/wall.err || { rc=$?; break; }
  echo "== new $i" && timeout -k 10 120 python scripts/msv_overhead.py >> $O/wall_new.jsonl 2>> $O/wall.err || { rc=$?; break; }
done
for which in new base; do
  [ $rc = 0 ] || break
  if [ $which = base ]; then export DN_SHAMIR_LIB="$BASE_LIB"; else unset DN_SHAMIR_LIB; fi
  echo "== rocprof $which" && (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_ab_$which -o run --output-format csv -- python3 "$R/scripts/mt_draw_rate.py" > "$R/$O/mt_draw_rate_$which.json" 2> "$R/$O/rocprof_$which.err") || rc=$?
  find /tmp/prof_ab_$which -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$which.csv \;
done
unset DN_SHAMIR_LIB
cat $O/wall_base.jsonl $O/wall_new.jsonl 2>/dev/null
for f in base new; do echo "-- $f"; cut -c1-600 $O/mt_draw_rate_$f.json 2>/dev/null; echo; grep -i "mt_\|split_kernel" $O/kernel_stats_$f.csv 2>/dev/null | cut -c1-160; done
echo "== rc $rc"
exit $rc
