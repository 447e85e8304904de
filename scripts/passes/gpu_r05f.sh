#!/bin/bash
# Round-5 pass f: the headline line on one GPU's shard of the 2^24 vector at
# N = 8 / 4 / 2 (bench.py --log2n 21 / 22 / 23, headline only), two processes
# each, with every chunked share block probed.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05f}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for r in 1 2; do
  for lg in 21 22 23; do
    echo "== log2n $lg run $r" && timeout -k 10 200 python bench.py --log2n $lg --rows 0 --config4 0 --config5 0 --cpu-budget 0 > $O/bench_$lg.$r.json 2>> $O/bench.err || { rc=$?; break 2; }
    python3 -c "
import json;d=json.load(open('$O/bench_$lg.$r.json'));r=d['roofline'];pl=r['placement']
print('%.3e'%d['value'],round(d['ms_per_step'],4),'split',[round(x,4) for x in pl['split_ms']],'recon',round(d['kernels']['reconstruct_ms'],4),'probed',[round(x or 0,2) for x in pl['probed_write_TBps']],d['parity']['all_ranks_ok'])"
  done
done
echo "== rc $rc"
exit $rc
