#!/bin/bash
# Round-6 pass b: mask accumulate A/B (product vs small-tile variants, alternating
# processes), then the mask GPU tests (small-tile path through the tuning build).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
T=${TAG:-r06b}
O=gpurun_out/$T
mkdir -p $O
rc=0
for round in 1 2; do
  for lib in libdn_shamir.so ab/libdn_shamir_mask6.so ab/libdn_shamir_mask7.so ab/libdn_shamir_mask5.so; do
    DN_SHAMIR_LIB=delta-node_amd/lib/$lib timeout -k 10 120 python scripts/mask_ab.py >> $O/mask_ab.jsonl 2>> $O/mask_ab.err || { rc=$?; echo "== $lib rc $rc"; tail -3 $O/mask_ab.err; exit $rc; }
  done
done
cut -c1-220 $O/mask_ab.jsonl
echo "== pytest mask" && timeout -k 10 600 python -u -m pytest tests/test_gpu_mask.py -x -v --timeout 300 --timeout-method thread > $O/pytest_mask.log 2>&1 || rc=$?
tail -2 $O/pytest_mask.log
echo "== rc $rc"
exit $rc
