#!/bin/bash
# Round-5 pass ab: the N = 8 shard's workload on one GPU (bench.py --log2n 21,
# the default line otherwise trimmed to the headline rows), three runs, HEAD.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05ab}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for r in 1 2 3; do
  echo "== 2^21 $r" && timeout -k 10 240 python bench.py --log2n 21 --rows 0 --config4 0 --config5 0 --cold 0 --cpu-budget 2 > $O/b21_$r.json 2> $O/b21_$r.err || { rc=$?; tail -3 $O/b21_$r.err; break; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['value']/1e9, d['ms_per_step'], r['avg_launch_ms'], r['frac'], d['kernels']['reconstruct_ms'], d['parity'])" $O/b21_$r.json
done
echo "== rc $rc"
exit $rc
