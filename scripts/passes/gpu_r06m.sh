#!/bin/bash
# Round-6 pass m: product (final state by the last substream + speculation)
# vs HEAD~1 (final-state wave, no speculation), alternating processes:
# loops and lone calls at 2^20 / 2^24 (scripts/msv_loop.py), incl. lone calls
# into pooled share blocks.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06m}
O=gpurun_out/$T
mkdir -p $O
rc=0
for round in 1 2 3 4; do
  for lib in libdn_shamir.so ab/libdn_shamir_HEAD.so; do
    SIZES=20,24 DN_SHAMIR_LIB=delta-node_amd/lib/$lib timeout -k 10 120 python scripts/msv_loop.py >> $O/msv_loop.jsonl 2>> $O/msv_loop.err || { rc=$?; echo "== $lib rc $rc"; tail -3 $O/msv_loop.err; exit $rc; }
  done
done
cut -c1-700 $O/msv_loop.jsonl
echo "== rc $rc"
exit $rc
