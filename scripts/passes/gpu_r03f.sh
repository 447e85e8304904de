#!/bin/bash
# Round-3 pass 6: fused-store cache policy on the current fused kernel (same
# process, tuning library), then SQ counter passes of the current AES encrypt,
# fused MT draw + split and ChaCha split.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r03f}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== mt aux" && AUXES=2,0,16,1,18 timeout -k 10 240 python scripts/mt_aux_probe.py > $O/mt_aux.json 2> $O/mt_aux.err || rc=$?
cut -c1-400 $O/mt_aux.json
if [ $rc = 0 ]; then TAG=${TAG:-r03f}_pmc KINDS="aes msv prng" bash scripts/passes/gpu_pmc_r03.sh || rc=$?; fi
echo "== rc $rc"
exit $rc
