#!/bin/bash
# Round-5 pass d: the runtime direct level in chunks (DN_MT_RT_CHUNKS, tuning
# build) — equivalence tests, then make_shares_vec at 2^24 per chunk count in
# alternating processes (scripts/msv_ab.py under the tuning library).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05d}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "chunks or runtime_direct or 2e24_digest_and" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head -5; exit $rc; }
TL="$R/delta-node_amd/lib/libdn_shamir_tuning.so"
for r in 1 2; do
  for c in ${CHUNKS:-1 2 3 4}; do
    echo "== round $r chunks $c" && DN_SHAMIR_LIB="$TL" DN_MT_RT_CHUNKS=$c timeout -k 10 120 python scripts/msv_ab.py > $O/ab_c${c}_r$r.json 2>> $O/ab.err || { rc=$?; break 2; }
    python3 -c "import json;d=json.load(open('$O/ab_c${c}_r$r.json'));print($c, [round(x,4) for x in d['2^24_ms_by_block']], d['equal_draw_then_split'])"
  done
done
echo "== rc $rc"
exit $rc
