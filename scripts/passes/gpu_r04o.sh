#!/bin/bash
# Round-4 pass o: generation-phase stagger probe (tuning build DN_MT_STAGGER),
# kernel trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04o}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== stagger probe"
cd /tmp && DN_SHAMIR_LIB=$R/delta-node_amd/lib/libdn_shamir_tuning.so timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/mts -o run --output-format csv -- python3 "$R/scripts/mt_stagger_probe.py" > "$R/$O/stagger.json" 2> "$R/$O/stagger.err" || rc=$?
cd "$R"
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/stagger.err; exit $rc; }
python3 scripts/mt_gen_probe_summary.py /tmp/mts $O/stagger.json > $O/stagger_summary.json || rc=$?
python3 -c "import json;d=json.load(open('$O/stagger_summary.json'));[print('stagger',r['stagger'],round(r['gen_us_median'],1),[round(x) for x in r['gen_us']]) for r in d['rows']]"
echo "== rc $rc"
exit $rc
