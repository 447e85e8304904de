#!/bin/bash
# Round-4 final pass: smoke, the whole GPU suite, make_shares_vec per-call
# times, the default bench line, the rocprof kernel summary of the same bench
# command, then the HBM traffic passes (separate --pmc runs, kernel trace
# only) over scripts/prof_kernels.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r04final}
mkdir -p $O
export TMPDIR=/tmp
TAG=${TAG:-r04final} bash scripts/passes/gpu_r04m.sh || exit $?
TAG=${TAG:-r04final}_pmc SRC="round 4 (final pass)" bash scripts/passes/gpu_pmc_r04.sh
