#!/bin/bash
# Round-2 PMC passes (one counter group per pass, kernel-trace only) over
# scripts/prof_kernels.py: split, reconstruct, fused draw+split, mask row.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/pmc_r02"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/pmc_fetch -o run --output-format csv -- python3 "$R/scripts/prof_kernels.py" > "$R/gpurun_out/pmc_r02/fetch.log" 2>&1 \
&& timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/pmc_write -o run --output-format csv -- python3 "$R/scripts/prof_kernels.py" > "$R/gpurun_out/pmc_r02/write.log" 2>&1 \
&& timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace -d /tmp/pmc_req -o run --output-format csv -- python3 "$R/scripts/prof_kernels.py" > "$R/gpurun_out/pmc_r02/req.log" 2>&1 \
&& for d in pmc_fetch pmc_write pmc_req; do find /tmp/$d -name "*counter_collection.csv" -exec cp {} "$R/gpurun_out/pmc_r02/$d.csv" \; ; done \
&& cd "$R" && python3 scripts/pmc_summary.py gpurun_out/pmc_r02 gpurun_out/pmc_r02/pmc_traffic.json > /dev/null \
&& echo "== pmc done"
