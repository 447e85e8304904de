#!/bin/bash
# Round-5 pass g: wave schedules (DN_TILE_MAP 0/2/3) on the blocks of one
# process at 2^21 and 2^24 (do slow blocks split faster under another
# schedule?), then the shard line (bench.py --log2n 21) with 12 probe tries
# for small blocks.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05g}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== sweep" && SIZES=21,24 MAPS=0,2,3 CAPS=0,1024 REPS=6 DN_SHAMIR_LIB="$R/delta-node_amd/lib/libdn_shamir_tuning.so" timeout -k 10 400 python scripts/small_shard_probe.py > $O/small_shard.jsonl 2> $O/small_shard.err || rc=$?
python3 -c "
import json
for l in open('$O/small_shard.jsonl'):
    d=json.loads(l); print(d['log2n'],d['cap'],d['map'],[round(x,4) for x in d['split_ms']],[round(x,4) for x in d['recon_ms']],round(d['step_ms'],4),'%.3e'%d['elems_per_s'],d['roundtrip'])"
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/small_shard.err; exit $rc; }
for r in 1 2; do
  echo "== log2n 21 run $r" && timeout -k 10 200 python bench.py --log2n 21 --rows 0 --config4 0 --config5 0 --cpu-budget 0 > $O/bench_21.$r.json 2>> $O/bench.err || { rc=$?; break; }
  python3 -c "
import json;d=json.load(open('$O/bench_21.$r.json'));r=d['roofline'];pl=r['placement']
print('%.3e'%d['value'],round(d['ms_per_step'],4),'split',[round(x,4) for x in pl['split_ms']],'recon',round(d['kernels']['reconstruct_ms'],4),'probed',[round(x or 0,2) for x in pl['probed_write_TBps']],pl['pool']['rejected'])"
done
echo "== rc $rc"
exit $rc
