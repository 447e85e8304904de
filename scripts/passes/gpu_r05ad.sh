#!/bin/bash
# Round-5 pass ad: the probe's tries for share blocks of 1 GiB and up (4 within
# 24 GiB, the default, vs 8 within 48 GiB) on the headline bench line,
# alternating processes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05ad}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for r in 1 2 3; do
  for k in 48,4,24 48,8,48; do
    echo "== tries $k run $r" && timeout -k 10 300 python scripts/bench_tries.py $k --rows 0 --config4 0 --config5 0 --cold 0 --cpu-budget 0 > $O/b24_${k}_$r.json 2> $O/b24_${k}_$r.err || { rc=$?; tail -3 $O/b24_${k}_$r.err; break 2; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; p=r['placement']; print(d['value']/1e9, d['ms_per_step'], r['avg_launch_ms'], [round(x,4) for x in p['split_ms']], [round(x,2) for x in p['probed_write_TBps']], p['pool']['probed'], p['pool']['rejected'])" $O/b24_${k}_$r.json
  done
done
echo "== rc $rc"
exit $rc
