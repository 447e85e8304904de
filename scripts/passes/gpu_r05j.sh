#!/bin/bash
# Round-5 pass j: the AES envelope with base64+hex by LDS lookups — AES GPU
# tests, then the encrypt kernel A/B against the SWAR build (lib/ab/
# libdn_shamir_aesswar.so), alternating processes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05j}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest aes" && timeout -k 10 300 python -u -m pytest tests/test_gpu_aes.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_aes.log 2>&1 || rc=$?
tail -2 $O/pytest_aes.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest_aes.log | head -5; exit $rc; }
TAG=${TAG:-r05j} VARIANTS="${VARIANTS:-aesswar}" bash scripts/passes/gpu_r05i.sh || rc=$?
exit $rc
