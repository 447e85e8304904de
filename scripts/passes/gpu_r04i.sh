#!/bin/bash
# Round-4 pass i: (1) tools/vmm_reuse_probe — does a VMM share block alias
# live hipMalloc memory after an earlier block was freed (four free
# strategies); (2) the generation kernel's anatomy on share blocks
# (scripts/mt_gen_probe.py under the tuning library, kernel trace).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04i}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== vmm reuse" && timeout -k 10 200 ./tools/vmm_reuse_probe > $O/vmm_reuse.txt 2>&1 || rc=$?
grep -E "^mode|overlaps [1-9]|bad_block_bytes [1-9]|bad_seg_bytes [1-9]|->" $O/vmm_reuse.txt | head -40
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
echo "== debug (share_block, torch.empty, share_block_sync, chunked_nopool) x3" && TRIALS=12 timeout -k 10 240 python scripts/msv_block_debug.py > $O/debug.jsonl 2> $O/debug.err || rc=$?
python3 -c "
import json
for l in open('$O/debug.jsonl'):
    d=json.loads(l)
    if 'trial' in d: print(d['trial'],d['kind'],d['ptr'],'overlap',d['torch_segments_overlapping'],'diff rows',sorted(d['diff']),sorted(d['diff_after_sync']),d['pool'])
"
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/debug.err; exit $rc; }
echo "== mt gen probe"
cd /tmp && DN_SHAMIR_LIB=$R/delta-node_amd/lib/libdn_shamir_tuning.so timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/mtg -o run --output-format csv -- python3 "$R/scripts/mt_gen_probe.py" > "$R/$O/mt_gen_probe.json" 2> "$R/$O/mt_gen_probe.err" || rc=$?
cd "$R"
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/mt_gen_probe.err; exit $rc; }
python3 scripts/mt_gen_probe_summary.py /tmp/mtg $O/mt_gen_probe.json > $O/mt_gen_summary.json || rc=$?
python3 -c "import json;d=json.load(open('$O/mt_gen_summary.json'));[print(r['block'],r['kind'],'back',r['back'],'probe',r['probe'],'fg',r.get('fwd_groups'),round(r['gen_us_median'],1)) for r in d['rows']];print('jump',d['jump_us_median'])"
grep -o '"fwd_groups_equal_output.*' $O/mt_gen_probe.json
echo "== rc $rc"
exit $rc
