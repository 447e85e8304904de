#!/bin/bash
# Round-4 pass d: MT parity tests with the job tables resident on the device
# (per-call copy = head + W_idx + row 0), make_shares_vec's GPU timeline and
# per-call wall time, then the fused kernel's store policy and generation /
# emission probes on 2 MiB-chunk share blocks (tuning library).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04d}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== test" && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_memory.py -x -v -m gpu -k "mt or fused or draw or memory or block or shares_vec or digest or shard" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
echo "== msv trace"
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/msvtr -o run --output-format csv -- python3 "$R/scripts/msv_trace.py" 12 16 24 > "$R/$O/msv_trace.json" 2> "$R/$O/msv_trace.err" || rc=$?
cd "$R"
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
mkdir -p $O/msvtr && find /tmp/msvtr -name "*.csv" -exec cp {} $O/msvtr/ \;
python3 scripts/msv_trace_summary.py $O/msvtr 24 > $O/msv_timeline.json || true
echo "== msv overhead" && timeout -k 10 200 python scripts/msv_overhead.py > $O/msv_overhead.json 2>&1 || rc=$?
tail -1 $O/msv_overhead.json | cut -c1-800
[ $rc -ne 0 ] && { echo "== rc $rc"; exit $rc; }
echo "== aux probe chunk" && OUTS=chunk PROBE=1 timeout -k 10 300 python scripts/mt_aux_probe.py > $O/mt_aux_chunk.json 2> $O/mt_aux_chunk.err || rc=$?
cut -c1-900 $O/mt_aux_chunk.json
echo "== rc $rc"
exit $rc
