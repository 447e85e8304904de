#!/bin/bash
# Mask row: its gpu tests, then the bench row alone (ROWS=mask).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "mask or agg or e2e" --timeout 120 --timeout-method thread > gpurun_out/pytest_mask.log 2>&1 \
&& ROWS=mask timeout -k 10 200 python scripts/rows_probe.py > gpurun_out/mask_row.json 2> gpurun_out/mask_row.err
rc=$?
tail -3 gpurun_out/pytest_mask.log
exit $rc
