#!/bin/bash
# Round-5 pass a: smoke, the whole GPU suite (stream-ordered share-block pool,
# the timed path's 2^24 reference digest), the VMM reuse probe with kernel
# traffic (modes 5-7), then the default bench line (cold first-call row).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05a}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || rc=$?
tail -1 $O/smoke.log
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -5; exit $rc; }
echo "== vmm reuse probe (kernel modes)" && timeout -k 10 120 ./tools/vmm_reuse_probe 7 > $O/vmm_reuse_kernel.txt 2>&1 || rc=$?
grep "bad cycles" $O/vmm_reuse_kernel.txt
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/vmm_reuse_kernel.txt; exit $rc; }
echo "== bench" && timeout -k 10 700 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || rc=$?
cut -c1-400 $O/bench_n1.json
python3 -c "
import json;d=json.load(open('$O/bench_n1.json'));print('parity',d['parity']);print('cold',json.dumps(d['rows']['draw_split'].get('cold'))[:1500])" || true
echo "== rc $rc"
exit $rc
