#!/bin/bash
# Round-5 pass n: two-pass AES decrypt — AES GPU tests, then decrypt A/B
# against the one-pass build (lib/ab/libdn_shamir_aesdec1p.so).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05n}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest aes+e2e" && timeout -k 10 400 python -u -m pytest tests/test_gpu_aes.py tests/test_gpu_e2e.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head -5; exit $rc; }
TAG=${TAG:-r05n} VARIANTS=aesdec1p bash scripts/passes/gpu_r05i.sh || rc=$?
exit $rc
