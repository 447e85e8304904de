#!/bin/bash
# Round-2 session-2 GPU pass: split-level MT jumps + MiMC7 squaring.
# Parity tests of the touched paths, MT draw rate, bench rows, placement
# layout A/B, rocprof kernel stats of the MT draw.  Each GPU step has its own
# time limit; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out/r02c
export TMPDIR=/tmp
O=gpurun_out/r02c
echo "== tests" && timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_mimc7.py -x -q -m gpu -k "mt or draw or config4 or sharded or fused or digest or reference or gpu_matches or gpu_vs" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
&& echo "== mt rate" && timeout -k 10 200 python scripts/mt_draw_rate.py > $O/mt_draw_rate.json 2> $O/mt_draw_rate.err \
&& echo "== rows" && ROWS=draw_split,rows timeout -k 10 300 python scripts/rows_probe.py > $O/rows.json 2> $O/rows.err \
&& echo "== place" && timeout -k 10 200 ./tools/place_probe 4 > $O/place_il.jsonl 2> $O/place_il.err \
&& echo "== rocprof" && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_mt -o run --output-format csv -- python3 "$R/scripts/mt_draw_rate.py" > "$R/$O/rocprof_mt.log" 2>&1 \
&& cd "$R" && mkdir -p $O/prof_mt && find /tmp/prof_mt -name "*stats.csv" -exec cp {} $O/prof_mt/ \; \
&& echo "== done"
rc=$?
tail -3 $O/pytest.log 2>/dev/null
cat $O/mt_draw_rate.json 2>/dev/null
exit $rc
