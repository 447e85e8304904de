#!/bin/bash
# Round-5 pass k: AES tests + encrypt A/B (pipelined vs not, vs the LDS-hex
# build of pass j), then the MT generation builtin change A/B against the
# build before it (scripts/ab_msv.sh: MT/fused parity tests, make_shares_vec
# per call alternating, kernel stats of the draw under each library).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
rc=0
TAG=r05k VARIANTS="aespipe0 aeshexnc" bash scripts/passes/gpu_r05j.sh || rc=$?
[ $rc -ne 0 ] && exit $rc
TAG=r05k_mt BASE=preMT bash scripts/ab_msv.sh || rc=$?
exit $rc
