#!/bin/bash
# Round-5 pass i: AES hex-envelope encrypt kernel, product vs variants
# (lib/ab/libdn_shamir_<NAME>.so), alternating processes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05i}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for r in 1 2; do
  for v in product ${VARIANTS:-aescoal}; do
    if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
    echo "== $v $r" && timeout -k 10 120 python scripts/aes_enc_time.py >> $O/aes.jsonl 2>> $O/aes.err || { rc=$?; break 2; }
    tail -1 $O/aes.jsonl
  done
done
echo "== rc $rc"
exit $rc
