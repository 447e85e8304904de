#!/bin/bash
# Round-3 pass o: where the MT generation kernels spend their time — kernel
# stats of scripts/mt_draw_rate.py (tuning library, all substreams forward)
# with DN_MT_PROBE = 0 (full), 1 (no emission: generation only), 2 (no
# generation: emission from a stale ring).  Outputs of probes 1 / 2 are
# garbage by design; only the times are read.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03o}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for probe in 0 1 2; do
  [ $rc = 0 ] || break
  echo "== probe $probe"
  export DN_SHAMIR_LIB=$R/delta-node_amd/lib/libdn_shamir_tuning.so DN_MT_BACK=0 DN_MT_PROBE=$probe
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_probe_$probe -o run --output-format csv -- python3 "$R/scripts/mt_draw_rate.py" > "$R/$O/mt_draw_rate_$probe.json" 2> "$R/$O/rocprof_$probe.err") || rc=$?
  find /tmp/prof_probe_$probe -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$probe.csv \;
  grep -h "mt_gen" $O/kernel_stats_$probe.csv | cut -d, -f1-4
done
echo "== rc $rc"
exit $rc
