#!/bin/bash
# Round-5 pass ak: the N = 8 / 4 / 2 shards' workloads on one GPU (bench.py
# --log2n 21 / 22 / 23, headline rows only), HEAD, two runs each.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05ak}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for r in 1 2; do
  for L in 21 22 23; do
    echo "== 2^$L $r" && timeout -k 10 300 python bench.py --log2n $L --rows 0 --config4 0 --config5 0 --cold 0 --cpu-budget 0 > $O/b${L}_$r.json 2> $O/b${L}_$r.err || { rc=$?; tail -3 $O/b${L}_$r.err; break 2; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; p=r['placement']; print(d['value']/1e9, d['ms_per_step'], r['avg_launch_ms'], round(r['frac'],3), d['kernels']['reconstruct_ms'], [round(x,2) for x in p['probed_write_TBps']], d['parity']['all_ranks_ok'])" $O/b${L}_$r.json
  done
done
echo "== rc $rc"
exit $rc
