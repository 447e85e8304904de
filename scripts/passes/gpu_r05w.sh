#!/bin/bash
# Round-5 pass w: AES encrypt/decrypt kernels, product (three keystream
# blocks interleaved, DN_AES_NB=3) vs NB = 1 and 2, alternating processes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05w}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for r in 1 2 3; do
  for v in product ${VARIANTS:-nb1 nb2}; do
    if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
    echo "== $v $r" && timeout -k 10 120 python scripts/aes_enc_time.py >> $O/aes.jsonl 2>> $O/aes.err || { rc=$?; break 2; }
    tail -1 $O/aes.jsonl
  done
done
echo "== rc $rc"
exit $rc
