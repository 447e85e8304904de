#!/bin/bash
# Round-4 pass z: the allocator's probe in the split's write order
# (dn_block_probe_rows): memory tests, then the bench line (its placement
# field shows each block's probed rate next to its split).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04z}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_memory.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
echo "== bench" && timeout -k 10 500 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || rc=$?
python3 -c "
import json;d=json.load(open('$O/bench_n1.json'));r=d['roofline'];pl=r['placement']
print('value',d['value'],'frac',round(r['frac'],4),'split',[round(x,3) for x in pl['split_ms']],'probed',[round(x,2) for x in pl['probed_write_TBps']],pl['pool'])
print('fused',d['rows']['draw_split']['fused_ms_by_buffer'],d['rows']['draw_split']['fused_ms_by_size'])"
echo "== rc $rc"
exit $rc
