#!/bin/bash
# Round-5 pass b: cold-call anatomy — VMM mapping cost per chunk size and
# thread count (tools/vmm_alloc_cost), the split's placement on larger chunks
# (scripts/chunk_size_probe.py), and the reuse probe with B at A's address.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05b}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== vmm alloc cost" && timeout -k 10 180 ./tools/vmm_alloc_cost > $O/vmm_alloc_cost.jsonl 2>&1 || rc=$?
cat $O/vmm_alloc_cost.jsonl | cut -c1-300
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
echo "== vmm reuse probe (kernel modes)" && timeout -k 10 120 ./tools/vmm_reuse_probe 7 > $O/vmm_reuse_kernel.txt 2>&1 || rc=$?
grep -E "bad cycles|same_va 1" $O/vmm_reuse_kernel.txt
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
echo "== chunk size probe" && timeout -k 10 400 python scripts/chunk_size_probe.py > $O/chunk_size.jsonl 2> $O/chunk_size.err || rc=$?
tail -1 $O/chunk_size.jsonl
echo "== rc $rc"
exit $rc
