#!/bin/bash
# Anatomy of the jump levels (tuning build, DN_MT_JUMP_PROBE): kernel stats of
# scripts/mt_draw_rate.py with the full jump (0), without the Horner steps (1:
# stream stepping + table only) and without the stream stepping of split
# levels' parts (2).  Timing only: probes 1 and 2 give wrong windows.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-jump_probe}
mkdir -p $O
export TMPDIR=/tmp
export DN_SHAMIR_LIB="$R/delta-node_amd/lib/libdn_shamir_tuning.so"
rc=0
for p in ${PROBES:-0 1 2}; do
  [ $rc = 0 ] || break
  echo "== probe $p" && (cd /tmp && DN_MT_JUMP_PROBE=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/jp_$p -o run --output-format csv -- python3 "$R/scripts/mt_draw_rate.py" > "$R/$O/rate_$p.json" 2> "$R/$O/rocprof_$p.err") || rc=$?
  find /tmp/jp_$p -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$p.csv \;
  grep -i "jump\|combine" $O/kernel_stats_$p.csv | cut -d, -f1-4 | cut -c1-140
done
echo "== rc $rc"
exit $rc
