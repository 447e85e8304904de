#!/bin/bash
# Round-3 pass u: level-B jump part count (tuning build DN_MT_PARTS_B; 0 =
# product heuristic, P = 4 at 2^24 with backward generation): kernel stats of
# scripts/mt_draw_rate.py per setting (jump kernels + combines per draw).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03u}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for P in 0 1 2 8 0; do
  [ $rc = 0 ] || break
  echo "== parts $P"
  export DN_SHAMIR_LIB=$R/delta-node_amd/lib/libdn_shamir_tuning.so DN_MT_PARTS_B=$P
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_parts_$P -o run --output-format csv -- python3 "$R/scripts/mt_draw_rate.py" > "$R/$O/mt_draw_rate_$P.json" 2> "$R/$O/rocprof_$P.err") || rc=$?
  find /tmp/prof_parts_$P -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$P.csv \;
  rm -rf /tmp/prof_parts_$P
  python3 - "$O/kernel_stats_$P.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
gen = sum(int(r["Calls"]) for r in rows if "mt_gen_kernel" in r["Name"])
jt = sum(float(r["TotalDurationNs"]) for r in rows if "mt_jump" in r["Name"] or "mt_combine" in r["Name"])
print({r["Name"][29:62]: (r["Calls"], round(float(r["AverageNs"]) / 1e3, 1)) for r in rows if "mt_" in r["Name"]})
print("jumps+combines per draw (us):", round(jt / max(gen, 1) / 1e3, 1))
PY
done
echo "== rc $rc"
exit $rc
