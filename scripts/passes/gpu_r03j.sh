#!/bin/bash
# Round-3 pass j: device-PRNG split (ChaCha20 / 12 / 8, 3-of-5, 2^24) kernel
# time by grid cap (tuning library, DN_GRID_CAP; default = 16384 workgroups,
# one tile per wave), two passes in alternation.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03j}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for rep in 1 2; do
  for cap in ${CAPS:-0 256 512 1024 1536 2048 4096 8192}; do
    [ $rc = 0 ] || break
    echo "== cap $cap rep $rep"
    if [ $cap = 0 ]; then
      timeout -k 10 120 python scripts/prng_ab.py > $O/tmp.json 2>> $O/prng.err || rc=$?
    else
      DN_SHAMIR_LIB=$R/delta-node_amd/lib/libdn_shamir_tuning.so DN_GRID_CAP=$cap timeout -k 10 120 python scripts/prng_ab.py > $O/tmp.json 2>> $O/prng.err || rc=$?
    fi
    [ $rc = 0 ] && python3 -c "import json,sys; d=json.load(open('$O/tmp.json')); d['grid_cap']=$cap; print(json.dumps(d))" >> $O/prng_gridcap.jsonl
  done
done
cat $O/prng_gridcap.jsonl
echo "== rc $rc"
exit $rc
