#!/bin/bash
# Round-5 pass c: embedded MT jump rows + 16 MiB chunks + fast-class probe bar:
# memory and parity GPU tests, the cold first call (both modes), then the
# default bench line.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05c}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest memory+parity" && timeout -k 10 600 python -u -m pytest tests/test_gpu_memory.py tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -5; exit $rc; }
for m in e2e phases e2e; do
  echo "== cold $m" && timeout -k 10 120 python scripts/cold_call.py --mode $m >> $O/cold.jsonl 2>> $O/cold.err || rc=$?
  tail -1 $O/cold.jsonl | cut -c1-700
  [ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/cold.err; exit $rc; }
done
echo "== bench" && timeout -k 10 700 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || rc=$?
python3 -c "
import json;d=json.load(open('$O/bench_n1.json'));r=d['roofline'];pl=r['placement']
print('value',d['value'],'frac',round(r['frac'],4),'split',[round(x,3) for x in pl['split_ms']],'probed',[round(x,2) for x in pl['probed_write_TBps']],pl['pool'])
print('parity',d['parity']); ds=d['rows']['draw_split']
print('fused',ds['fused_ms_by_buffer'],ds['fused_ms_by_size']); print('cold',json.dumps(ds.get('cold'))[:900])" || true
echo "== rc $rc"
exit $rc
