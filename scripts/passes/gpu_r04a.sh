#!/bin/bash
# Round-4 pass a: the GPU suite (new full-size reference pins, the 8-rank
# driver-command rehearsal, the all-elements config-4 check), the share-block
# placement experiment (scripts/block_probe.py), and a kernel + copy trace of
# make_shares_vec at 2^12 / 2^16 / 2^24 (scripts/msv_trace.py).
# A test failure (rc 1) lets the measurements run; a crash, abort or time
# limit ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04a}
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
rc=0
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
tail -3 $O/pytest_gpu.log
if fatal $rc; then echo "== stop rc $rc"; exit $rc; fi
prc=$rc
echo "== block probe"
timeout -k 10 400 python -u scripts/block_probe.py 5 > $O/block_probe.jsonl 2> $O/block_probe.err || rc=$?
tail -1 $O/block_probe.jsonl | cut -c1-1500
if [ $rc -ne 0 ] && [ $rc -ne $prc ]; then echo "== stop rc $rc"; tail -5 $O/block_probe.err; exit $rc; fi
echo "== msv trace"
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/msvtr -o run --output-format csv -- python3 "$R/scripts/msv_trace.py" 12 16 24 > "$R/$O/msv_trace.json" 2> "$R/$O/msv_trace.err" || rc=$?
cd "$R"
if [ $rc -eq 0 ] || [ $rc -eq $prc ]; then
  mkdir -p $O/msvtr && find /tmp/msvtr -name "*.csv" -exec cp {} $O/msvtr/ \;
  python3 scripts/msv_trace_summary.py $O/msvtr 24 > $O/msv_timeline.json || true
  cat $O/msv_trace.json
fi
echo "== rc $rc (pytest $prc)"
exit $rc
