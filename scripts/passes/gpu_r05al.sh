#!/bin/bash
# Round-5 pass al: the first share block of a class under 1 GiB as the fastest
# of 4 tries (PROBE_FIRST_SMALL, HEAD) vs of 2, on the 2^21 shard's line,
# alternating processes; the memory GPU tests first.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05al}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest" && timeout -k 10 300 python -u -m pytest tests/test_gpu_memory.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -1 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head -5; exit $rc; }
for r in 1 2 3; do
  for f in 4 2; do
    echo "== first $f run $r" && timeout -k 10 300 python scripts/bench_tries.py 48,8,48,$f --log2n 21 --rows 0 --config4 0 --config5 0 --cold 0 --cpu-budget 0 > $O/b21_f${f}_$r.json 2> $O/b21_f${f}_$r.err || { rc=$?; tail -3 $O/b21_f${f}_$r.err; break 2; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; p=r['placement']; print(d['value']/1e9, d['ms_per_step'], r['avg_launch_ms'], [round(x,4) for x in p['split_ms']], [round(x,2) for x in p['probed_write_TBps']], p['pool']['probed'])" $O/b21_f${f}_$r.json
  done
done
echo "== rc $rc"
exit $rc
