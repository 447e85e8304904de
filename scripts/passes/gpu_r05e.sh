#!/bin/bash
# Round-5 pass e: the headline step on the 2/4/8-GPU shards (2^23/22/21) on
# one GPU — grid caps and wave schedules (scripts/small_shard_probe.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05e}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== sweep" && DN_SHAMIR_LIB="$R/delta-node_amd/lib/libdn_shamir_tuning.so" timeout -k 10 400 python scripts/small_shard_probe.py > $O/small_shard.jsonl 2> $O/small_shard.err || rc=$?
python3 -c "
import json
for l in open('$O/small_shard.jsonl'):
    d=json.loads(l); print(d['log2n'],d['cap'],d['map'],[round(x,4) for x in d['split_ms']],[round(x,4) for x in d['recon_ms']],round(d['step_ms'],4),'%.3e'%d['elems_per_s'],d['roundtrip'])"
echo "== rc $rc"
exit $rc
