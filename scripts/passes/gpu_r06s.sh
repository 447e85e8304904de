#!/bin/bash
# Round-6 pass s: the generation's wave priority beside the speculated level
# (DN_MT_GEN_PRIO, tuning build): 2^24 loops and lone calls (scripts/msv_loop.py)
# at priorities 0 / 1 / 2 / 3, alternating rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06s}
O=gpurun_out/$T
mkdir -p $O
rc=0
for round in 1 2 3; do
  for P in 0 1 2 3; do
    echo "{\"round\": $round, \"prio\": $P}" >> $O/prio.jsonl
    SIZES=24 DN_MT_GEN_PRIO=$P DN_SHAMIR_LIB=delta-node_amd/lib/libdn_shamir_tuning.so timeout -k 10 120 python scripts/msv_loop.py >> $O/prio.jsonl 2>> $O/prio.err || { rc=$?; echo "== rc $rc"; tail -3 $O/prio.err; exit $rc; }
  done
done
cut -c1-330 $O/prio.jsonl
echo "== rc $rc"
exit $rc
