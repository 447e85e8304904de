#!/bin/bash
# Round-6 pass j: speculated levels vs their part count (tuning build,
# DN_MT_PARTS_B = parts per jump of the 2^24 direct level; more, shorter parts
# let CUs freed early in the generation's tail take more of the level):
# 2^24 loops (scripts/msv_loop.py) with and without speculation, alternating.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06j}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rc=0
for round in 1 2; do
  for P in 4 8 16; do
    for SP in 1 0; do
      echo "{\"round\": $round, \"parts\": $P, \"spec\": $SP}" >> $O/parts.jsonl
      SIZES=24 DN_MT_PARTS_B=$P DN_MT_SPEC=$SP DN_SHAMIR_LIB=delta-node_amd/lib/libdn_shamir_tuning.so timeout -k 10 120 python scripts/msv_loop.py >> $O/parts.jsonl 2>> $O/parts.err || { rc=$?; echo "== rc $rc"; tail -3 $O/parts.err; exit $rc; }
    done
  done
done
cut -c1-300 $O/parts.jsonl
echo "== rc $rc"
exit $rc
