#!/bin/bash
# MT jump-table layout A/B: lib/libdn_shamir_prev.so (comparison build) vs the library as built;
# per-size make_shares_vec walls (alternating twice), kernel trace of the new build, MT parity tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/mtab2
mkdir -p $O
export TMPDIR=/tmp
PREV=$R/delta-node_amd/lib/libdn_shamir_prev.so
echo "== tests" && timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q -m gpu -k "mt or draw or fused or sharded or config4 or concurrent or boundaries" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
&& echo "== walls" && timeout -k 10 100 python scripts/msv_overhead.py > $O/new1.json 2>> $O/err.log \
&& DN_SHAMIR_LIB=$PREV timeout -k 10 100 python scripts/msv_overhead.py > $O/prev1.json 2>> $O/err.log \
&& timeout -k 10 100 python scripts/msv_overhead.py > $O/new2.json 2>> $O/err.log \
&& DN_SHAMIR_LIB=$PREV timeout -k 10 100 python scripts/msv_overhead.py > $O/prev2.json 2>> $O/err.log \
&& echo "== trace" && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_ab2 -o run --output-format csv -- python3 "$R/scripts/msv_overhead.py" > "$R/$O/rocprof.log" 2>&1 \
&& cd "$R" && find /tmp/prof_ab2 -name "*kernel_trace.csv" -exec cp {} $O/ \; \
&& echo "== done"
rc=$?
tail -2 $O/pytest.log; for f in new1 prev1 new2 prev2; do echo $f; cat $O/$f.json; done
exit $rc
