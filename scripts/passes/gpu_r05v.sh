#!/bin/bash
# Round-5 pass v: where the ~40 us between back-to-back make_shares_vec calls
# goes: kernel + memory-copy traces of the default pooled output and of a
# caller's block passed as out=, and the host time of the pool alone.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${TAG:-r05v}
mkdir -p $O
export TMPDIR=/tmp
rc=0
for m in default caller; do
  echo "== trace $m" && cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/msvgap_$m -o run --output-format csv -- python3 "$R/scripts/msv_loop_gaps.py" 24 $m > "$R/$O/trace_wall_$m.json" 2> "$R/$O/trace_$m.err" || rc=$?
  cd "$R"
  [ $rc -ne 0 ] && { echo "== rc $rc"; tail -3 $O/trace_$m.err; exit $rc; }
  python3 scripts/msv_loop_gaps.py --summary /tmp/msvgap_$m > $O/gaps_$m.json && cut -c1-400 $O/gaps_$m.json
done
for m in phases default caller; do
  timeout -k 10 120 python scripts/msv_loop_gaps.py 24 $m >> $O/walls.jsonl 2>> $O/walls.err || { rc=$?; break; }
  tail -1 $O/walls.jsonl
done
echo "== rc $rc"
exit $rc
