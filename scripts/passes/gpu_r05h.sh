#!/bin/bash
# Round-5 pass h: wave schedule A/B on the bench line itself (tuning library,
# DN_TILE_MAP 0 = cyclic vs 3 = coop, split and reconstruct), alternating
# processes, at 2^24 and 2^21; bench with two events per step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05h}
mkdir -p $O
export TMPDIR=/tmp
rc=0
TL="$R/delta-node_amd/lib/libdn_shamir_tuning.so"
for r in 1 2; do
  for lg in 24 21; do
    for m in 0 3; do
      echo "== log2n $lg map $m run $r" && DN_SHAMIR_LIB="$TL" DN_TILE_MAP=$m timeout -k 10 200 python bench.py --log2n $lg --rows 0 --config4 0 --config5 0 --cpu-budget 0 > $O/bench_${lg}_m$m.$r.json 2>> $O/bench.err || { rc=$?; break 3; }
      python3 -c "
import json;d=json.load(open('$O/bench_${lg}_m$m.$r.json'));r=d['roofline'];pl=r['placement']
print('%.4e'%d['value'],round(d['ms_per_step'],4),'split',round(r['avg_launch_ms'],4),[round(x,4) for x in pl['split_ms']],'recon',round(d['kernels']['reconstruct_ms'],4),'probed',[round(x or 0,2) for x in pl['probed_write_TBps']],d['parity']['all_ranks_ok'])"
    done
  done
done
echo "== rc $rc"
exit $rc
