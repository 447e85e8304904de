#!/bin/bash
# Round-4 pass s: generation anatomy of the two-wave kernel forced at 2^24 vs
# the one-wave kernel (tuning build: DN_MT_PC_FORCE, DN_MT_PROBE), kernel trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04s}
mkdir -p $O
export TMPDIR=/tmp
rc=0
cd /tmp && DN_SHAMIR_LIB=$R/delta-node_amd/lib/libdn_shamir_tuning.so BACKS=1 PCS=0,1 NO_FG=1 REPS=4 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/mtpc -o run --output-format csv -- python3 "$R/scripts/mt_gen_probe.py" > "$R/$O/pc_probe.json" 2> "$R/$O/pc_probe.err" || rc=$?
cd "$R"
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/pc_probe.err; exit $rc; }
python3 scripts/mt_gen_probe_summary.py /tmp/mtpc $O/pc_probe.json > $O/pc_summary.json || rc=$?
python3 -c "import json;d=json.load(open('$O/pc_summary.json'));[print(r['kind'],'pc',r['pc'],'probe',r['probe'],round(r['gen_us_median'],1)) for r in d['rows']]"
echo "== rc $rc"
exit $rc
