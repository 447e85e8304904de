#!/bin/bash
# Round-4 spread: the default bench line again on this box, then the
# per-GPU shard sizes of the strong-scaling lines (2^23 / 2^22 / 2^21: the
# 2-, 4- and 8-GPU shards of the 2^24 vector) on one GPU, headline only.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04spread}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== bench" && timeout -k 10 500 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || rc=$?
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/bench_n1.err; exit $rc; }
for lg in 23 22 21; do
  echo "== shard 2^$lg" && timeout -k 10 200 python bench.py --log2n $lg --rows 0 --config4 0 --config5 0 --cpu-budget 0 --steps 50 > $O/bench_2e$lg.json 2> $O/bench_2e$lg.err || rc=$?
  [ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/bench_2e$lg.err; exit $rc; }
done
python3 -c "
import json
for f in ['bench_n1','bench_2e23','bench_2e22','bench_2e21']:
    d=json.load(open('$O/'+f+'.json'));r=d['roofline']
    print(f,'value',round(d['value']/1e9,3),'e9 ms/step',round(d['ms_per_step'],4),'split frac',round(r['frac'],4),'blocks',[round(x,3) for x in r['placement']['split_ms']] if r.get('placement') else None)
"
echo "== rc $rc"
exit $rc
