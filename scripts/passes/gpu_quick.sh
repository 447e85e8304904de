#!/bin/bash
# Quick GPU pass: selected parity tests (PYTEST_K) and one bench row (ROWS) via scripts/rows_probe.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/quick
mkdir -p $O
export TMPDIR=/tmp
echo "== tests" && timeout -k 10 500 python -u -m pytest ${PYTEST_FILES:-tests} -x -q -m gpu -k "${PYTEST_K:-mt}" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
&& echo "== rows" && timeout -k 10 300 python scripts/rows_probe.py > $O/rows.json 2> $O/rows.err \
&& echo "== done"
rc=$?
tail -2 $O/pytest.log; cut -c1-3000 $O/rows.json
exit $rc
