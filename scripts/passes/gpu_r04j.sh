#!/bin/bash
# Round-4 pass j: the share-block fix (freed VMM ranges retired, never
# re-reserved): scripts/msv_block_debug.py (12 trials, the r04i pattern
# that corrupted every new block at a freed block's address), then the
# memory and MT parity GPU tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04j}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== debug" && TRIALS=12 timeout -k 10 240 python scripts/msv_block_debug.py > $O/debug.jsonl 2> $O/debug.err || rc=$?
python3 -c "
import json
for l in open('$O/debug.jsonl'):
    d=json.loads(l)
    if 'trial' in d: print(d['trial'],d['kind'],d['ptr'],'diff rows',sorted(d['diff']),sorted(d['diff_after_sync']),d['pool'])
"
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -5 $O/debug.err; exit $rc; }
echo "== tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_memory.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -3 $O/pytest.log
echo "== rc $rc"
exit $rc
