#!/bin/bash
# Round-4 pass t: the two-wave kernel with an LDS-only barrier (pc_barrier)
# and separate producer / consumer loops: MT parity tests, then its anatomy
# forced at 2^24 against the one-wave kernel (tuning build), then msv_ab.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04t}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_memory.py -x -q -m gpu -k "mt or draw or fused or sharded or config4 or digest or shares_vec" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
cd /tmp && DN_SHAMIR_LIB=$R/delta-node_amd/lib/libdn_shamir_tuning.so BACKS=1 PCS=0,1 NO_FG=1 REPS=4 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/mtpc -o run --output-format csv -- python3 "$R/scripts/mt_gen_probe.py" > "$R/$O/pc_probe.json" 2> "$R/$O/pc_probe.err" || rc=$?
cd "$R"
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/pc_probe.err; exit $rc; }
python3 scripts/mt_gen_probe_summary.py /tmp/mtpc $O/pc_probe.json > $O/pc_summary.json || rc=$?
python3 -c "import json;d=json.load(open('$O/pc_summary.json'));[print(r['kind'],'pc',r['pc'],'probe',r['probe'],round(r['gen_us_median'],1)) for r in d['rows']]"
echo "== msv_ab" && timeout -k 10 200 python scripts/msv_ab.py > $O/ab_new.jsonl 2> $O/ab.err || rc=$?
cut -c1-420 $O/ab_new.jsonl
echo "== rc $rc"
exit $rc
