#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only) + tuning sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/pmc_fetch -o run --output-format csv -- python3 "$R/scripts/prof_kernels.py" > "$R/gpurun_out/pmc_fetch.log" 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/pmc_write -o run --output-format csv -- python3 "$R/scripts/prof_kernels.py" > "$R/gpurun_out/pmc_write.log" 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace -d /tmp/pmc_req -o run --output-format csv -- python3 "$R/scripts/prof_kernels.py" > "$R/gpurun_out/pmc_req.log" 2>&1 \
&& mkdir -p "$R/gpurun_out/pmc_$TAG" && for d in pmc_fetch pmc_write pmc_req; do find /tmp/$d -name "*counter_collection.csv" -exec cp {} "$R/gpurun_out/pmc_$TAG/$d.csv" \; ; done \
&& cd "$R" && timeout -k 10 300 python scripts/tune_kernels.py > gpurun_out/tune.jsonl 2> gpurun_out/tune.err \
&& echo "== prof done"
rc=$?
ls gpurun_out/pmc_$TAG 2>/dev/null
cat gpurun_out/tune.jsonl 2>/dev/null
exit $rc
