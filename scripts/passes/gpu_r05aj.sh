#!/bin/bash
# Round-5 pass aj: the headline split with the next quarter's loads ahead of
# the current quarter's stores (DN_SPLIT_PF=1, variant splitpf): parity GPU
# tests on the variant, then the headline bench line (trimmed rows),
# alternating processes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05aj}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== pytest splitpf" && DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_splitpf.so" timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
tail -1 $O/pytest.log
[ $rc -ne 0 ] && { echo "== rc $rc"; grep -E "FAILED|Error" $O/pytest.log | head -5; exit $rc; }
for r in 1 2 3; do
  for v in product splitpf; do
    if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
    timeout -k 10 300 python bench.py --rows 0 --config4 0 --config5 0 --cold 0 --cpu-budget 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { rc=$?; tail -3 $O/b_${v}_$r.err; break 2; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; p=r['placement']; print(sys.argv[2], d['value']/1e9, d['ms_per_step'], r['avg_launch_ms'], [round(x,4) for x in p['split_ms']], [round(x,3) for x in p['split_frac_of_ceiling']], d['kernels']['reconstruct_ms'])" $O/b_${v}_$r.json $v
  done
done
echo "== rc $rc"
exit $rc
