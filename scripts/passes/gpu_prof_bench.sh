#!/bin/bash
# rocprofv3 kernel summary of the default bench command (no CPU baseline: its
# worker processes would each load the profiler).  CSV under gpurun_out/prof_bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/prof_bench"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_bench -o run --output-format csv -- python3 "$R/bench.py" --cpu-budget 0 > "$R/gpurun_out/bench_prof.json" 2> "$R/gpurun_out/bench_prof.err" \
&& cp -r /tmp/prof_bench/. "$R/gpurun_out/prof_bench/"
