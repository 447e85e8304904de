#!/bin/bash
# A/B of make_shares_vec (fused MT19937 draw + split) per-call wall time:
# the baseline library lib/ab/libdn_shamir_${BASE}.so (make ab REF=...) and the
# in-tree library, alternating processes, then the kernel stats of the new
# one and the MT / fused parity tests.  Each GPU step has its own time limit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-abmsv}
mkdir -p $O
export TMPDIR=/tmp
BASE_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_${BASE:-HEAD}.so"
rc=0
for i in 1 2; do
  echo "== base $i" && DN_SHAMIR_LIB="$BASE_LIB" timeout -k 10 120 python scripts/msv_overhead.py >> $O/wall_base.jsonl 2>> $O/wall.err || { rc=$?; break; }
  echo "== new $i" && timeout -k 10 120 python scripts/msv_overhead.py >> $O/wall_new.jsonl 2>> $O/wall.err || { rc=$?; break; }
done
if [ $rc = 0 ]; then
  echo "== rocprof new" && (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_ab -o run --output-format csv -- python3 "$R/scripts/msv_overhead.py" > "$R/$O/rocprof.log" 2>&1) || rc=$?
  find /tmp/prof_ab -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
fi
if [ $rc = 0 ]; then
  echo "== rocprof base" && (cd /tmp && DN_SHAMIR_LIB="$BASE_LIB" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_ab_base -o run --output-format csv -- python3 "$R/scripts/msv_overhead.py" > "$R/$O/rocprof_base.log" 2>&1) || rc=$?
  find /tmp/prof_ab_base -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_base.csv \;
fi
if [ $rc = 0 ] && [ -z "$NOTEST" ]; then
  echo "== tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q -m gpu -k "mt or draw or fused or sharded or config4 or digest" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
  tail -2 $O/pytest.log
fi
cat $O/wall_base.jsonl $O/wall_new.jsonl
for f in kernel_stats_base kernel_stats; do echo "-- $f"; grep -i "mt_" $O/$f.csv 2>/dev/null | cut -c1-160; done
echo "== rc $rc"
exit $rc
