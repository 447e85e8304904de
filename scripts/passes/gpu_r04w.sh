#!/bin/bash
# Round-4 pass w: ChaCha split occupancy A/B (launch bounds 6 = in-tree, 5, 4
# waves per SIMD): scripts/prng_ab.py alternating, two rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04w2}
mkdir -p $O
rc=0
for i in 1 2; do
  for v in new w5 w4; do
    echo "== prng $v $i"
    if [ $v = new ]; then timeout -k 10 120 python scripts/prng_ab.py >> $O/prng_$v.jsonl 2>> $O/prng.err || rc=$?
    else DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so" timeout -k 10 120 python scripts/prng_ab.py >> $O/prng_$v.jsonl 2>> $O/prng.err || rc=$?; fi
    [ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/prng.err; exit $rc; }
  done
done
for v in new w5 w4; do python3 -c "
import json
for l in open('$O/prng_$v.jsonl'):
    d=json.loads(l); print('$v', round(d['chacha20_ms'],4), round(d['chacha12_ms'],4), round(d['chacha8_ms'],4), d['chacha20_roundtrip'])"; done
echo "== rc $rc"
exit $rc
