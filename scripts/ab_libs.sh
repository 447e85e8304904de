#!/bin/bash
# A/B of the MT19937 device draw over several product libraries: the in-tree
# library ("new") and lib/ab/libdn_shamir_<V>.so for each V in $VARIANTS
# (make ab REF=... / make variant NAME=...).  First the MT / fused parity tests
# of the in-tree library and of every variant, then make_shares_vec per-call
# wall time (processes alternating over the libraries, $ROUNDS rounds), then the
# kernel stats of scripts/mt_draw_rate.py under each library.  Each GPU step
# has its own time limit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-ablibs}
mkdir -p $O
export TMPDIR=/tmp
VARIANTS=${VARIANTS:-HEAD}
ALL="new $VARIANTS"
# run "$@" with DN_SHAMIR_LIB naming variant $V (unset for the in-tree library)
with_lib() { local v=$1; shift; if [ "$v" = new ]; then env -u DN_SHAMIR_LIB "$@"; else DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so" "$@"; fi; }
rc=0
for v in $ALL; do
  [ $rc = 0 ] || break
  [ -n "$NOTEST" ] && break
  [ "$v" = HEAD ] && continue
  echo "== tests $v" && with_lib $v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py \
      -x -q -m gpu -k "mt or draw or fused or sharded or config4 or digest" --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || rc=$?
  tail -1 $O/pytest_$v.log
done
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in $ALL; do
    [ $rc = 0 ] || break 2
    echo "== wall $v $i" && with_lib $v timeout -k 10 120 python scripts/msv_overhead.py >> $O/wall_$v.jsonl 2>> $O/wall.err || rc=$?
  done
done
for v in $ALL; do
  [ $rc = 0 ] || break
  echo "== rocprof $v" && (cd /tmp && with_lib $v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_ab_$v -o run --output-format csv -- python3 "$R/scripts/mt_draw_rate.py" > "$R/$O/mt_draw_rate_$v.json" 2> "$R/$O/rocprof_$v.err") || rc=$?
  find /tmp/prof_ab_$v -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$v.csv \;
done
for v in $ALL; do
  echo "-- $v"; cat $O/wall_$v.jsonl 2>/dev/null | cut -c1-300
  grep -i "mt_" $O/kernel_stats_$v.csv 2>/dev/null | cut -d, -f1-6 | cut -c1-150
done
echo "== rc $rc"
exit $rc
