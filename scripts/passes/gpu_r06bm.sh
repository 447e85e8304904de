#!/bin/bash
# Round 6: speculation beside small generations (DN_MT_BESIDE_MIN) — the
# speculation / parity / sharded GPU tests, then make_shares_vec loops and lone
# calls (scripts/msv_loop.py) alternating the product library with the build
# that never speculates beside a small generation (lib/ab/libdn_shamir_bmoff.so,
# make variant NAME=bmoff VFLAGS=-DDN_MT_BESIDE_MIN=2^62).
set -o pipefail
O=gpurun_out/${TAG:-bm}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=delta-node_amd/lib
for i in 1 2 3 4; do
  for v in $L/libdn_shamir.so $L/ab/libdn_shamir_bmoff.so; do
    SIZES=${SIZES:-12,14,16,17,18,20,21} DN_SHAMIR_LIB=$PWD/$v timeout -k 10 150 python scripts/msv_loop.py >> $O/msv_loop.jsonl 2>>$O/err.log || exit 1
  done
done
echo done
