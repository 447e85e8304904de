#!/bin/bash
# Round-5 pass u: make_shares_vec back to back (default pooled output): the
# GPU timeline's gaps between calls (kernel + memory-copy trace), then wall
# time per call, product vs the spin-wait variant (DN_MT_SPIN_SYNC=1),
# alternating processes, at 2^24 and 2^20.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05u}
mkdir -p $O
export TMPDIR=/tmp
rc=0
echo "== trace" && cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/msvgap -o run --output-format csv -- python3 "$R/scripts/msv_loop_gaps.py" 24 > "$R/$O/trace_wall.json" 2> "$R/$O/trace.err" || rc=$?
cd "$R"
[ $rc -ne 0 ] && { echo "== rc $rc"; tail -3 $O/trace.err; exit $rc; }
python3 scripts/msv_loop_gaps.py --summary /tmp/msvgap > $O/gaps.json && cut -c1-700 $O/gaps.json
for r in 1 2 3; do
  for L in 24 20; do
    for v in product spin; do
      if [ $v = product ]; then unset DN_SHAMIR_LIB; else export DN_SHAMIR_LIB="$R/delta-node_amd/lib/ab/libdn_shamir_$v.so"; fi
      timeout -k 10 120 python scripts/msv_loop_gaps.py $L >> $O/walls.jsonl 2>> $O/walls.err || { rc=$?; break 3; }
      tail -1 $O/walls.jsonl
    done
  done
done
echo "== rc $rc"
exit $rc
